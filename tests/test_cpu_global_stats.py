"""Global statistics of the batch-coupled losses over data-parallel ranks (SURVEY.md §8e option
ii) on CPU: the shard decomposition of oracle/global_stats.py (the restatement of the
csrc/loss.hip phase kernels) against the oracle's whole-batch ContrastRegionLoss /
ContrastEdgeLoss (modules/trainer.py:89-184): emulated shards in one process, and the real
world-2 gloo path through modules/parallel.py's all-reduce."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from oracle import global_stats as gs
from oracle import prng
from oracle import ref_torch as orc

THR, WEIGHT = 0.15, 1.5  # modules/trainer.py:357
# The reference (and the oracle) take these means / std / top-k means in float32; the shard
# sums are float64, so the two agree to float32 rounding of the statistics, not bitwise.
TOL = 1e-5


def _batch(n, hw, seed):
    mk = lambda name: torch.from_numpy(prng.uniform(seed, name, (n, 1, hw, hw), -1, 1))
    return mk("p"), mk("t"), mk("s")


def _sum(parts):
    return torch.stack(parts).sum(0)


def _rel(a, b):
    return abs(float(a) - float(b)) / max(abs(float(b)), 1e-12)


@pytest.mark.parametrize("split", [[4], [2, 2], [1, 3], [1, 1, 2]])
def test_sharded_losses_equal_whole_batch(split):
    p, t, s = _batch(sum(split), 32, 7)
    want_r = orc.contrast_region_loss(p, t, s, THR, WEIGHT)
    want_e = orc.contrast_edge_loss(p, t)
    cuts = torch.tensor([0] + split).cumsum(0).tolist()
    shards = [(p[a:b], t[a:b], s[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    got_r = gs.region_sharded(shards, THR, WEIGHT, _sum)
    got_e = gs.edge_sharded([(a, b) for a, b, _ in shards], _sum)
    assert _rel(got_r, want_r) < TOL, (float(got_r), float(want_r))
    assert _rel(got_e, want_e) < TOL, (float(got_e), float(want_e))


def test_edge_topk_with_ties():
    """Flat regions give many equal edge magnitudes: the k-th largest value is tied and the
    top-k mean takes only the missing count of the tied value (as torch.topk's values do)."""
    p = torch.zeros(2, 1, 32, 32)
    p[:, :, 8:24, 8:24] = 1.0
    t = torch.from_numpy(prng.uniform(3, "t", (2, 1, 32, 32), -1, 1))
    want = orc.contrast_edge_loss(p, t)
    got = gs.edge_sharded([(p[:1], t[:1]), (p[1:], t[1:])], _sum)
    assert _rel(got, want) < TOL


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    from conftest import ROOT
    sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd")]
    torch.set_num_threads(1)
    from modules import parallel
    try:
        parallel.init_from_env("gloo")
        p, t, s = _batch(4, 32, 11)
        a, b = parallel.shard(4)
        mine = [(p[a:b], t[a:b], s[a:b])]
        red = lambda parts: parallel.allreduce_sum_(parts[0].clone())
        r = gs.region_sharded(mine, THR, WEIGHT, red)
        e = gs.edge_sharded([(x, y) for x, y, _ in mine], red)
        q.put((rank, float(r), float(e)))
    except Exception as ex:  # noqa: BLE001
        q.put((rank, repr(ex), None))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def test_gloo_world2_global_loss_stats():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for pr in procs:
        pr.join(timeout=60)
    p, t, s = _batch(4, 32, 11)
    want_r = float(orc.contrast_region_loss(p, t, s, THR, WEIGHT))
    want_e = float(orc.contrast_edge_loss(p, t))
    for rank, r, e in res:
        assert e is not None, r
        assert _rel(r, want_r) < TOL and _rel(e, want_e) < TOL, (rank, r, want_r, e, want_e)
