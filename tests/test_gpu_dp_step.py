"""The product training step under data parallelism: CycleGANSystem.train_step (explicit schedule,
modules/trainer.py) in two processes sharing one GPU over gloo, against one process running the
whole batch.  This is the step that replaces the reference's nn.DataParallel training
(/root/reference/modules/trainer.py:307, 333-338, 447-525), with the batch-coupled loss terms
(trainer.py:126-128, 170-180) over the whole data-parallel batch by default.

What two ranks must reproduce (bs 4 at 64x64, 2 residual blocks with CBAM, cin 3, two steps):
  * step-0 loss terms: the mean over ranks of each rank's value equals the one-process value of
    the whole batch within 1e-5 relative (mean-type terms are shard means; ContrastRegion /
    ContrastEdge are computed over the whole batch on every rank);
  * the parameters after each step: the G and D gradients are all-reduced means of the shard
    gradients, so the replicas follow the whole-batch run.  Adam's first update is lr * sign(g),
    so an entry whose gradient is decided by rounding can move the other way: median |delta| <=
    1e-6, max <= 2 * lr * (steps taken);
  * every replica bit-identical (parallel.replicas_identical, and the checksums here);
  * ``--per_rank_loss_stats`` (losses.GLOBAL_STATS = False): each rank's step-0 terms equal a
    one-process run on that rank's shard alone (within 1e-5);
  * ``split_groups(2)`` (BASELINE config 5 on split GPU groups): a soft-tissue (cin 3) model on
    rank 0 and a lung (cin 2) model on rank 1, each bit-identical to its own one-process run.

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
N, HW, NB, STEPS, SEED, LR = 4, 64, 2, 2, 811, 2e-4


def _sd(shapes, seed):
    return {k: torch.from_numpy(v) for k, v in prng.init_state_dict(shapes, seed).items()}


def _system(cin):
    from modules.trainer import CycleGANSystem
    s = CycleGANSystem(cin, NB, True, lr=LR, device=DEV, init=False)
    seeds = prng.step_model_seeds(SEED + cin)
    gs, ds = orc.generator_param_shapes(cin, NB, True), orc.discriminator_param_shapes(1)
    s.G_A2B.load_state_dict(_sd(gs, seeds["G_A2B"]))
    s.G_B2A.load_state_dict(_sd(gs, seeds["G_B2A"]))
    s.D_A.load_state_dict(_sd(ds, seeds["D_A"]))
    s.D_B.load_state_dict(_sd(ds, seeds["D_B"]))
    return s


def _batch(step, cin):
    rA = torch.from_numpy(prng.uniform(SEED, f"A{step}", (N, 1, HW, HW), -1, 1))
    rB = torch.from_numpy(prng.uniform(SEED, f"B{step}", (N, 1, HW, HW), -1, 1))
    mk = torch.from_numpy(prng.bernoulli(SEED + cin, f"M{step}", (N, cin - 1, HW, HW), 0.3))
    return rA, rB, mk


def _run(cin, a, b, steps):
    """Train a fresh system on samples [a, b) of every step's batch; per step the loss terms
    and the three optimizers' flat parameters (host copies)."""
    s = _system(cin)
    rec = {"losses": [], "params": []}
    for i in range(steps):
        rA, rB, mk = (t[a:b].to(DEV) for t in _batch(i, cin))
        out = s.train_step(rA, rB, mk)
        rec["losses"].append({k: float(v) for k, v in out.items()})
        rec["params"].append([o.flat_p.detach().cpu().clone() for o in s.optimizers])
    return s, rec


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, world, port, mode, outdir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), DUCOSY_DEVICE_OVERRIDE="0", DUCOSY_DIST_BACKEND="gloo")
    import sys
    from conftest import ROOT
    sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd")]
    import torch.distributed as dist
    try:
        from modules import losses, parallel
        parallel.init_from_env()
        torch.cuda.set_device(0)
        cin = 3
        if mode == "per_rank":
            losses.GLOBAL_STATS = False
        if mode == "groups":
            gi, _ = parallel.split_groups(2)
            cin = (3, 2)[gi]
        a, b = parallel.shard(N)
        s, rec = _run(cin, a, b, STEPS if mode != "per_rank" else 1)
        flats = [o.flat_p for o in s.optimizers]
        rec.update(identical=parallel.replicas_identical(flats), checksums=parallel.replica_checksums(flats).cpu(),
                   shard=(a, b), cin=cin, world=parallel.world(), stats=losses.stats_mode())
        torch.save(rec, os.path.join(outdir, f"rank{rank}.pt"))
    except Exception as ex:  # noqa: BLE001
        import traceback
        torch.save({"error": repr(ex) + "\n" + traceback.format_exc()}, os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _launch(mode, tmp_path):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, str(tmp_path))) for r in range(2)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
        if pr.is_alive():
            pr.kill()
            pytest.fail(f"{mode}: a rank did not finish in 240 s")
    res = []
    for r in range(2):
        rec = torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=False)  # written by this test
        assert "error" not in rec, rec.get("error")
        res.append(rec)
    return res


def _rel(v, ref):
    return abs(v - ref) / max(abs(ref), 1e-12)


def _param_delta(got, want, bound, where):
    for k, (g, w) in enumerate(zip(got, want)):
        d = (g - w).abs()
        med, mx = float(d.median()), float(d.max())
        assert med <= 1e-6 and mx <= bound, (where, ("G", "D_A", "D_B")[k], med, mx)


def test_dp_two_ranks_equal_whole_batch(tmp_path):
    res = _launch("dp", tmp_path)
    _, full = _run(3, 0, N, STEPS)
    for r, rec in enumerate(res):
        assert rec["world"] == 2 and rec["shard"] == (2 * r, 2 * r + 2)
        assert rec["stats"] == "whole data-parallel batch"
        assert rec["identical"], "replicas_identical reported a diverged replica"
    assert torch.equal(res[0]["checksums"], res[1]["checksums"])
    # step 0: the rank mean of every term is the whole-batch value
    for k, v in full["losses"][0].items():
        m = sum(rec["losses"][0][k] for rec in res) / 2
        assert _rel(m, v) <= 1e-5, (k, m, v, [rec["losses"][0][k] for rec in res])
    # later steps follow from parameters that agree to Adam's sign-flip bound
    for k, v in full["losses"][1].items():
        m = sum(rec["losses"][1][k] for rec in res) / 2
        assert abs(m - v) <= 1e-3 * max(abs(v), abs(full["losses"][0][k]), 1e-2), (k, m, v)
    for i in range(STEPS):
        for rec in res:
            _param_delta(rec["params"][i], full["params"][i], 2 * LR * (i + 1) + 1e-7, f"step {i}")


def test_dp_per_rank_loss_stats_equal_shard_runs(tmp_path):
    res = _launch("per_rank", tmp_path)
    for r, rec in enumerate(res):
        assert rec["stats"] == "per rank (--per_rank_loss_stats)" and rec["identical"]
        _, shard_run = _run(3, 2 * r, 2 * r + 2, 1)
        for k, v in shard_run["losses"][0].items():
            assert _rel(rec["losses"][0][k], v) <= 1e-5, (r, k, rec["losses"][0][k], v)


def test_split_groups_soft_and_lung_equal_own_runs(tmp_path):
    res = _launch("groups", tmp_path)
    for r, rec in enumerate(res):
        assert rec["world"] == 1 and rec["cin"] == (3, 2)[r] and rec["shard"] == (0, N)
        _, own = _run(rec["cin"], 0, N, STEPS)
        for i in range(STEPS):
            assert rec["losses"][i] == own["losses"][i], (r, i, rec["losses"][i], own["losses"][i])
            for g, w in zip(rec["params"][i], own["params"][i]):
                assert torch.equal(g, w), (r, i, float((g - w).abs().max()))
