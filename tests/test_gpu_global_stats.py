"""Global statistics of the batch-coupled losses over data-parallel ranks (SURVEY.md §8e option
ii) on the GPU, through the C-ABI phase functions of csrc/loss.hip:
  * emulated ranks in lockstep on one device (partials summed between the phases, as the
    all-reduce would) give the loss of the WHOLE batch — equal to the one-call path on the full
    batch and to the oracle — and each shard's gradient is its slice of the whole-batch gradient;
  * the ops-level wrappers with one rank equal the one-call path;
  * two real processes (gloo, one GPU) through modules/losses.py's global_stats switch."""
import ctypes
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from oracle import prng
from oracle import ref_torch as orc

pytestmark = pytest.mark.gpu
DEV = "cuda"
THR, WEIGHT = 0.15, 1.5  # modules/trainer.py:357


def _batch(n, hw, seed):
    mk = lambda name: torch.from_numpy(prng.uniform(seed, name, (n, 1, hw, hw), -1, 1))
    return mk("p"), mk("t"), mk("s")


def _rel(a, b):
    return abs(float(a) - float(b)) / max(abs(float(b)), 1e-12)


def _relmax(a, b):
    return float((a - b).abs().max() / b.abs().max())


class _Shard:
    """One emulated rank: its slice and its own workspace / partial buffers."""

    def __init__(self, ops, lib, p, t, s):
        self.p, self.t, self.s = p.contiguous(), t.contiguous(), s.contiguous()
        self.N, _, self.H, self.W = p.shape
        nb = lib.query("dcs_loss_workspace_size", self.N, self.H, self.W)
        self.ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
        self.red = torch.zeros(9, dtype=torch.float64, device=DEV)
        self.hist = torch.empty(512, dtype=torch.int32, device=DEV)
        self.out = torch.empty(1, device=DEV)
        self.grad = torch.empty_like(self.p)
        self.ops, self.lib = ops, lib

    def call(self, fn, *args):
        self.lib.call(fn, *args, self.ops._p(self.ws), self.ws.numel(), self.ops._stream())


def _allsum(shards, get, set_):
    tot = sum(get(sh) for sh in shards)
    for sh in shards:
        set_(sh, tot.clone())


def _region_lockstep(shards):
    P = shards[0].ops._p
    for sh in shards:
        sh.call("dcs_loss_contrast_region_partial", P(sh.p), P(sh.t), P(sh.s), sh.N, sh.H, sh.W, THR, P(sh.red))
    _allsum(shards, lambda sh: sh.red, lambda sh, v: sh.red.copy_(v))
    for sh in shards:
        sh.call("dcs_loss_contrast_region_finish", P(sh.p), sh.N, sh.H, sh.W, WEIGHT, P(sh.red), 1.0, P(sh.out),
                P(sh.grad))


def _edge_lockstep(shards):
    P = shards[0].ops._p
    for sh in shards:
        sh.call("dcs_loss_contrast_edge_partial", P(sh.p), P(sh.t), sh.N, sh.H, sh.W, P(sh.red))
    _allsum(shards, lambda sh: sh.red[:5], lambda sh, v: sh.red[:5].copy_(v))
    for ps in range(4):
        for sh in shards:
            sh.call("dcs_loss_contrast_edge_hist", sh.N, sh.H, sh.W, ps, P(sh.red), P(sh.hist))
        _allsum(shards, lambda sh: sh.hist, lambda sh, v: sh.hist.copy_(v))
        for sh in shards:
            sh.call("dcs_loss_contrast_edge_select", ps, P(sh.hist))
    for sh in shards:
        sh.call("dcs_loss_contrast_edge_topk", sh.N, sh.H, sh.W, P(sh.red))
    _allsum(shards, lambda sh: sh.red[5:9], lambda sh, v: sh.red[5:9].copy_(v))
    for sh in shards:
        sh.call("dcs_loss_contrast_edge_finish", P(sh.p), sh.N, sh.H, sh.W, P(sh.red), 1.0, P(sh.out), P(sh.grad))


@pytest.fixture
def hip():
    from modules.hip import lib, ops
    return ops, lib


@pytest.mark.parametrize("split", [[2, 2], [1, 3], [4]])
def test_lockstep_shards_equal_whole_batch(hip, split):
    ops, lib = hip
    p, t, s = _batch(sum(split), 64, 21)
    pd, td, sd = p.to(DEV), t.to(DEV), s.to(DEV)
    vr, gr = ops.loss_contrast_region(pd, td, sd, THR, WEIGHT, True)
    ve, ge = ops.loss_contrast_edge(pd, td, True)
    cuts = torch.tensor([0] + split).cumsum(0).tolist()
    mk = lambda: [_Shard(ops, lib, pd[a:b], td[a:b], sd[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    shr = mk()
    _region_lockstep(shr)
    she = mk()
    _edge_lockstep(she)
    torch.cuda.synchronize()
    for sh in shr:
        assert _rel(sh.out, vr) < 1e-6, (float(sh.out), float(vr))
    for sh in she:
        assert _rel(sh.out, ve) < 1e-6, (float(sh.out), float(ve))
    assert _relmax(torch.cat([sh.grad for sh in shr]), gr) < 1e-5
    assert _relmax(torch.cat([sh.grad for sh in she]), ge) < 1e-5
    # pinned to the oracle's whole-batch losses (float32 statistics in the reference)
    assert _rel(shr[0].out, orc.contrast_region_loss(p, t, s, THR, WEIGHT)) < 1e-5
    assert _rel(she[0].out, orc.contrast_edge_loss(p, t)) < 1e-5


def test_ops_global_one_rank_equals_one_call(hip):
    ops, _ = hip
    p, t, s = (x.to(DEV) for x in _batch(2, 64, 22))
    ident = lambda x: x
    vr, gr = ops.loss_contrast_region(p, t, s, THR, WEIGHT, True)
    wr, hr = ops.loss_contrast_region_global(p, t, s, THR, WEIGHT, ident, 1.0, True)
    ve, ge = ops.loss_contrast_edge(p, t, True)
    we, he = ops.loss_contrast_edge_global(p, t, ident, 1.0, True)
    assert float(wr) == float(vr) and float(we) == float(ve)
    assert _relmax(hr, gr) < 1e-6 and _relmax(he, ge) < 1e-6


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), DUCOSY_DEVICE_OVERRIDE="0", DUCOSY_DIST_BACKEND="gloo")
    import sys
    from conftest import ROOT
    sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd")]
    try:
        from modules import losses, parallel
        parallel.init_from_env()
        torch.cuda.set_device(0)
        p, t, s = _batch(4, 64, 23)
        a, b = parallel.shard(4)
        out = []
        for mod, args in ((losses.ContrastRegionLoss(THR, WEIGHT, global_stats=True), (t, s)),
                          (losses.ContrastEdgeLoss(global_stats=True), (t,))):
            x = p[a:b].to(DEV).requires_grad_(True)
            v = mod(x, *[y[a:b].to(DEV) for y in args])
            v.backward()
            out.append((float(v), x.grad.detach().cpu()))
        q.put((rank, out))
    except Exception as ex:  # noqa: BLE001
        q.put((rank, repr(ex)))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def test_two_processes_gloo_global_stats(hip):
    ops, _ = hip
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for pr in procs:
        pr.join(timeout=60)
    p, t, s = (x.to(DEV) for x in _batch(4, 64, 23))
    full = [ops.loss_contrast_region(p, t, s, THR, WEIGHT, True), ops.loss_contrast_edge(p, t, True)]
    for r in (0, 1):
        assert isinstance(res[r], list), res[r]
        for (v, g), (fv, fg) in zip(res[r], full):
            assert _rel(v, fv) < 1e-6, (r, v, float(fv))
            # grad_scale = world: the DP all-reduce-mean of these equals the whole-batch gradient
            want = fg[2 * r:2 * r + 2].cpu()
            assert _relmax(g / 2, want) < 1e-5
