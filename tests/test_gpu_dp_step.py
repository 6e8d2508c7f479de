"""The product training step under data parallelism: CycleGANSystem.train_step (explicit schedule,
modules/trainer.py) in two processes sharing one GPU over gloo, against one process running the
whole batch.  This is the step that replaces the reference's nn.DataParallel training
(/root/reference/modules/trainer.py:307, 333-338, 447-525), with the batch-coupled loss terms
(trainer.py:126-128, 170-180) over the whole data-parallel batch by default.

What two ranks must reproduce (bs 4 at 64x64 with 2 residual blocks, and BASELINE config 4's
per-rank size: bs 8 per rank at 512x512 with 9 blocks against one process at bs 16; CBAM, cin 3,
two steps):
  * step-0 loss terms: the mean over ranks of each rank's value equals the one-process value of
    the whole batch within 1e-5 relative (mean-type terms are shard means; ContrastRegion /
    ContrastEdge are computed over the whole batch on every rank);
  * step-0 gradients: each optimizer's flat gradient after the all-reduce, as Adam receives it
    (FusedAdam.flat_g at step()), equals the whole-batch run's within relative L2 1e-5 for G, D_A
    and D_B (at 512 x 512 in f16x3: 5e-4, see the config-4 test).  This is the check Adam's parameters cannot give: its first update is lr * sign(g),
    invariant to the gradient's scale, so an all-reduce that divided by w^2, or a wrong
    grad_scale on the batch-coupled terms, would pass a parameter comparison;
  * the parameters after each step: the replicas follow the whole-batch run up to Adam's sign
    flips of gradients decided by rounding: median |delta| <= 1e-6, max <= 2.5 * lr * (steps taken)
    (an Adam step moves an entry by about lr, a little more where the second gradient outweighs the
    first: measured 8.04e-4 after two steps at 512 x 512);
  * every replica bit-identical (parallel.replicas_identical, and the checksums here);
  * ``--per_rank_loss_stats`` (losses.GLOBAL_STATS = False): each rank's step-0 terms equal a
    one-process run on that rank's shard alone (within 1e-5), and the all-reduced gradient equals
    the mean of the two shard runs' gradients (relative L2 1e-5);
  * ``split_groups(2)`` (BASELINE config 5 on split GPU groups): a soft-tissue (cin 3) model on
    rank 0 and a lung (cin 2) model on rank 1, each bit-identical to its own one-process run, in
    the default operand mode and in config 5's fp16 MFMA mode.

The RCCL (backend "nccl") path runs the same code with another backend; it needs one GPU per rank
and is exercised by the driver's multi-GPU bench."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from oracle import prng
from oracle import ref_torch as orc

pytestmark = pytest.mark.gpu
DEV = "cuda"
STEPS, SEED, LR = 2, 811, 2e-4
SMALL = dict(n=4, hw=64, nb=2)    # whole batch, image size, residual blocks
FULL = dict(n=16, hw=512, nb=9)   # BASELINE config 4 per rank: bs 8 at 512x512, 9 blocks
GRAD_TOL = 1e-5


def _sd(shapes, seed):
    return {k: torch.from_numpy(v) for k, v in prng.init_state_dict(shapes, seed).items()}


def _system(cin, nb):
    from modules.trainer import CycleGANSystem
    s = CycleGANSystem(cin, nb, True, lr=LR, device=DEV, init=False)
    seeds = prng.step_model_seeds(SEED + cin)
    gs, ds = orc.generator_param_shapes(cin, nb, True), orc.discriminator_param_shapes(1)
    s.G_A2B.load_state_dict(_sd(gs, seeds["G_A2B"]))
    s.G_B2A.load_state_dict(_sd(gs, seeds["G_B2A"]))
    s.D_A.load_state_dict(_sd(ds, seeds["D_A"]))
    s.D_B.load_state_dict(_sd(ds, seeds["D_B"]))
    return s


def _batch(step, cin, n, hw):
    rA = torch.from_numpy(prng.uniform(SEED, f"A{step}", (n, 1, hw, hw), -1, 1))
    rB = torch.from_numpy(prng.uniform(SEED, f"B{step}", (n, 1, hw, hw), -1, 1))
    mk = torch.from_numpy(prng.bernoulli(SEED + cin, f"M{step}", (n, cin - 1, hw, hw), 0.3))
    return rA, rB, mk


def _record_grads(s, rec):
    """Wrap each optimizer's step() to keep a host copy of the flat gradient it is about to apply
    (after the data-parallel all-reduce): rec["grads"][step][optimizer]."""
    for k, opt in enumerate(s.optimizers):
        def step(closure=None, _opt=opt, _orig=opt.step, _k=k):
            rec["grads"][-1][_k] = _opt.flat_g.detach().cpu().clone()
            return _orig(closure)
        opt.step = step


def _run(cin, a, b, steps, cfg):
    """Train a fresh system on samples [a, b) of every step's batch; per step the loss terms, the
    three optimizers' applied flat gradients and their flat parameters after the step (host copies)."""
    s = _system(cin, cfg["nb"])
    rec = {"losses": [], "params": [], "grads": []}
    _record_grads(s, rec)
    for i in range(steps):
        rA, rB, mk = (t[a:b].to(DEV) for t in _batch(i, cin, cfg["n"], cfg["hw"]))
        rec["grads"].append([None] * 3)
        out = s.train_step(rA, rB, mk)
        rec["losses"].append({k: float(v) for k, v in out.items()})
        rec["params"].append([o.flat_p.detach().cpu().clone() for o in s.optimizers])
    return s, rec


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, world, port, mode, cfg, mma, outdir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), DUCOSY_DEVICE_OVERRIDE="0", DUCOSY_DIST_BACKEND="gloo")
    import sys
    from conftest import ROOT
    sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd")]
    import torch.distributed as dist
    try:
        from modules import losses, parallel
        from modules.hip import ops
        ops.set_mma(mma)
        parallel.init_from_env()
        torch.cuda.set_device(0)
        cin = 3
        if mode == "per_rank":
            losses.GLOBAL_STATS = False
        if mode == "groups":
            gi, _ = parallel.split_groups(2)
            cin = (3, 2)[gi]
        a, b = parallel.shard(cfg["n"])
        s, rec = _run(cin, a, b, STEPS if mode != "per_rank" else 1, cfg)
        flats = [o.flat_p for o in s.optimizers]
        rec.update(identical=parallel.replicas_identical(flats), checksums=parallel.replica_checksums(flats).cpu(),
                   shard=(a, b), cin=cin, world=parallel.world(), stats=losses.stats_mode(), mma=ops.get_mma())
        torch.save(rec, os.path.join(outdir, f"rank{rank}.pt"))
    except Exception as ex:  # noqa: BLE001
        import traceback
        torch.save({"error": repr(ex) + "\n" + traceback.format_exc()}, os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _launch(mode, tmp_path, cfg=SMALL, mma="f16x3", timeout=240):
    torch.cuda.empty_cache()  # the ranks share this GPU with the test process
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, cfg, mma, str(tmp_path))) for r in range(2)]
    for pr in procs:
        pr.start()
    try:
        for pr in procs:  # every rank gets the timeout before any is killed
            pr.join(timeout=timeout)
    finally:
        hung = [r for r, pr in enumerate(procs) if pr.is_alive()]
        for pr in procs:
            if pr.is_alive():
                pr.kill()
                pr.join(timeout=30)
    if hung:
        pytest.fail(f"{mode}: ranks {hung} did not finish in {timeout} s")
    res = []
    for r in range(2):
        rec = torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=False)  # written by this test
        assert "error" not in rec, rec.get("error")
        res.append(rec)
    return res


def _rel(v, ref):
    return abs(v - ref) / max(abs(ref), 1e-12)


def _rel_l2(got, ref):
    return float((got.double() - ref.double()).norm() / ref.double().norm().clamp_min(1e-30))


def _param_delta(got, want, bound, where, med_tol=1e-6):
    for k, (g, w) in enumerate(zip(got, want)):
        d = (g - w).abs()
        med, mx = float(d.median()), float(d.max())
        assert med <= med_tol and mx <= bound, (where, ("G", "D_A", "D_B")[k], med, mx)


def _param_slices(system):
    """(name, start, stop) of every parameter in each optimizer's flat buffer."""
    out = []
    for opt, models in zip(system.optimizers, ((("G_A2B", system.G_A2B), ("G_B2A", system.G_B2A)),
                                               (("D_A", system.D_A),), (("D_B", system.D_B),))):
        sl, off = [], 0
        for mname, m in models:
            for pname, p in m.named_parameters():
                sl.append((f"{mname}.{pname}", off, off + p.numel()))
                off += p.numel()
        assert off == opt.flat_g.numel()
        out.append(sl)
    return out


def _check_grads(got, want, where, slices=None, tol=GRAD_TOL):
    """Step-0 applied gradients of the three optimizers: relative L2 against the reference gradients
    (on failure, the parameters that carry most of the difference)."""
    errs = []
    for k, (g, w) in enumerate(zip(got, want)):
        assert g is not None and w is not None and float(w.norm()) > 0, (where, k)
        e = _rel_l2(g, w)
        errs.append(e)
        if e > tol and slices is not None:
            d2 = sorted(((float((g[a:b].double() - w[a:b].double()).norm()), _rel_l2(g[a:b], w[a:b]), nm)
                         for nm, a, b in slices[k]), reverse=True)[:8]
            print(f"{where}: {('G', 'D_A', 'D_B')[k]} rel L2 {e:.3e}; largest contributions (|diff|, rel, name):", d2)
        assert e <= tol, (where, ("G", "D_A", "D_B")[k], e)
    return errs


def _dp_vs_whole_batch(res, full, cfg, slices=None, grad_tol=GRAD_TOL, med_tol=1e-6):
    n = cfg["n"]
    for r, rec in enumerate(res):
        assert rec["world"] == 2 and rec["shard"] == (r * n // 2, (r + 1) * n // 2)
        assert rec["stats"] == "whole data-parallel batch"
        assert rec["identical"], "replicas_identical reported a diverged replica"
    assert torch.equal(res[0]["checksums"], res[1]["checksums"])
    # step 0: the rank mean of every term is the whole-batch value
    for k, v in full["losses"][0].items():
        m = sum(rec["losses"][0][k] for rec in res) / 2
        assert _rel(m, v) <= 1e-5, (k, m, v, [rec["losses"][0][k] for rec in res])
    # step 0: the gradient each rank applied is the whole-batch gradient (both ranks apply the same)
    for rec in res:
        for g0, g1 in zip(rec["grads"][0], res[0]["grads"][0]):
            assert torch.equal(g0, g1), "the ranks applied different gradients"
    errs = _check_grads(res[0]["grads"][0], full["grads"][0], "step 0", slices, grad_tol)
    print(f"dp {cfg}: step-0 applied-gradient rel L2 (G, D_A, D_B) = {errs}")
    # later steps follow from parameters that agree to Adam's sign-flip bound
    for k, v in full["losses"][1].items():
        m = sum(rec["losses"][1][k] for rec in res) / 2
        assert abs(m - v) <= 1e-3 * max(abs(v), abs(full["losses"][0][k]), 1e-2), (k, m, v)
    for i in range(STEPS):
        for rec in res:
            _param_delta(rec["params"][i], full["params"][i], 2.5 * LR * (i + 1), f"step {i}", med_tol)


def test_dp_two_ranks_equal_whole_batch(tmp_path):
    res = _launch("dp", tmp_path)
    s, full = _run(3, 0, SMALL["n"], STEPS, SMALL)
    _dp_vs_whole_batch(res, full, SMALL, _param_slices(s))


@pytest.mark.parametrize("mma", ["f32", "f16x3"])
def test_dp_two_ranks_equal_whole_batch_config4_size(tmp_path, mma):
    """BASELINE config 4's per-rank work: two ranks at bs 8, 512 x 512, 9 blocks, cin 3, against one
    process at bs 16 (the whole data-parallel batch).

    Exact f32 MFMA: the step-0 gradients within relative L2 1e-5, as at 64 x 64.  f16x3: the operands'
    power-of-two scales come from the max |value| of each call's whole tensor, so a rank's 24-image
    Generator call and the whole batch's 48-image call can round differently (at ~1e-7), and a
    rounding that moves a pre-activation across a ReLU kink changes that pixel's gradient by O(1)
    (scripts/diag/bign_stages.py: each call's fused head gradient equals the unfused path on its own
    inputs within 4e-7).  The bar there is 5e-4 (measured 1.0e-4 for G, 1.6e-4 for D_A): a mis-scaled
    all-reduce or grad_scale is still off by percent or more.  The parameters after the second Adam step
    then differ by a median 2.5e-6 (bar 1e-5; f32: 1e-6), each flipped first-step sign moving an entry
    by up to 2 lr."""
    from modules.hip import ops
    res = _launch("dp", tmp_path, FULL, mma=mma, timeout=600)
    prev = ops.get_mma()
    ops.set_mma(mma)
    try:
        s, full = _run(3, 0, FULL["n"], STEPS, FULL)
    finally:
        ops.set_mma(prev)
    slices = _param_slices(s)
    del s
    torch.cuda.empty_cache()
    _dp_vs_whole_batch(res, full, FULL, slices, *((1e-5, 1e-6) if mma == "f32" else (5e-4, 1e-5)))


def test_dp_per_rank_loss_stats_equal_shard_runs(tmp_path):
    res = _launch("per_rank", tmp_path)
    shard_grads = []
    for r, rec in enumerate(res):
        assert rec["stats"] == "per rank (--per_rank_loss_stats)" and rec["identical"]
        _, shard_run = _run(3, 2 * r, 2 * r + 2, 1, SMALL)
        shard_grads.append(shard_run["grads"][0])
        for k, v in shard_run["losses"][0].items():
            assert _rel(rec["losses"][0][k], v) <= 1e-5, (r, k, rec["losses"][0][k], v)
    mean = [(g0 + g1) / 2 for g0, g1 in zip(*shard_grads)]
    _check_grads(res[0]["grads"][0], mean, "per-rank statistics, step 0")


@pytest.mark.parametrize("mma", ["f16x3", "f16"])
def test_split_groups_soft_and_lung_equal_own_runs(tmp_path, mma):
    from modules.hip import ops
    res = _launch("groups", tmp_path, mma=mma)
    prev = ops.get_mma()
    ops.set_mma(mma)
    try:
        for r, rec in enumerate(res):
            assert rec["world"] == 1 and rec["cin"] == (3, 2)[r] and rec["shard"] == (0, SMALL["n"])
            assert rec["mma"] == mma
            _, own = _run(rec["cin"], 0, SMALL["n"], STEPS, SMALL)
            for i in range(STEPS):
                assert rec["losses"][i] == own["losses"][i], (r, i, rec["losses"][i], own["losses"][i])
                for g, w in zip(rec["params"][i], own["params"][i]):
                    assert torch.equal(g, w), (r, i, float((g - w).abs().max()))
    finally:
        ops.set_mma(prev)
