"""Data parallelism: one process per GPU, torch.distributed over RCCL (backend "nccl").

Replaces the reference's single-process nn.DataParallel (modules/trainer.py:333-338), which
scatters every G/D call over 8 GPUs, re-broadcasts all parameters per call and reduces
gradients to cuda:0.  Here each rank owns full replicas of G_A2B, G_B2A, D_A, D_B and its own
batch shard; per optimizer step the optimizer's flat gradient buffer (FusedAdam.flat_g: 91.6 MB
for the G pair, 11.05 MB per D at cin 3) is averaged over the replicas by ONE stream-ordered
all-reduce after the backward, stream-ordered on the compute stream.  The exchange is not
overlapped with the backward: RCCL's kernels on a queue of their own beside the backward's would
share compute-unit pairs with it, the condition of the two-queue hazard (Config 5),
for at most ~1 ms of a ~200 ms step.  Initial weights
are broadcast from the group's first rank once; ``replicas_identical`` checks after a run that
every replica still holds the same parameters (bench.py reports it).

Replica group: by default every rank of the job.  ``set_group`` narrows it to a sub-group, for
BASELINE config 5 on one node as split GPU groups (soft-tissue model on ranks 0..w/2-1, lung
model on ranks w/2..w-1, each group with its own collectives; ``split_groups``).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

_GROUP = None  # process group of this rank's replicas (None: the default group)


def _on():
    return dist.is_available() and dist.is_initialized()


def set_group(group) -> None:
    """Collectives, world() and rank() refer to ``group`` from now on (None: every rank)."""
    global _GROUP
    _GROUP = group


def group():
    return _GROUP


def world():
    return dist.get_world_size(_GROUP) if _on() else 1


def rank():
    return dist.get_rank(_GROUP) if _on() else 0


def init_from_env(backend: str = None):
    """Initialise the default process group from torchrun's env (RANK/WORLD_SIZE/MASTER_*).
    Returns (rank, world_size, local_rank).  No-op for a single process."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = local_device_index()
    if ws <= 1:
        return 0, 1, local
    if not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("DUCOSY_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size(), local


def split_groups(n_groups: int):
    """Cut the job into ``n_groups`` equal contiguous rank groups (every rank must call this).
    Returns (index of this rank's group, its process group) and makes it the replica group."""
    w, r = dist.get_world_size(), dist.get_rank()
    if w % n_groups:
        raise ValueError(f"world size {w} is not a multiple of {n_groups} groups")
    per = w // n_groups
    mine = None
    for gi in range(n_groups):
        pg = dist.new_group(list(range(gi * per, (gi + 1) * per)))
        if gi == r // per:
            mine = pg
    set_group(mine)
    return r // per, mine


def local_device_index() -> int:
    """GPU of this process: LOCAL_RANK (one process per GPU).  DUCOSY_DEVICE_OVERRIDE pins
    every rank to one device — for rehearsing the multi-process path on a single GPU with
    DUCOSY_DIST_BACKEND=gloo (RCCL does not allow two ranks on one device)."""
    o = os.environ.get("DUCOSY_DEVICE_OVERRIDE")
    return int(o) if o not in (None, "") else int(os.environ.get("LOCAL_RANK", "0"))


def broadcast_(flat: torch.Tensor, src: int = 0):
    """Broadcast from the replica group's rank ``src``."""
    if world() > 1:
        gsrc = dist.get_global_rank(_GROUP, src) if _GROUP is not None else src
        dist.broadcast(flat, gsrc, group=_GROUP)
    return flat


def _scale_(flat: torch.Tensor, s: float):
    if flat.is_cuda:
        from .hip import ops
        ops.scale_add_(flat, flat, s - 1.0)  # flat *= s on the device kernel
    else:
        flat.mul_(s)


def allreduce_mean_(flat: torch.Tensor):
    """In-place mean over the replicas of a flat gradient buffer (one collective)."""
    w = world()
    if w == 1:
        return flat
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=_GROUP)
    _scale_(flat, 1.0 / w)
    return flat


def allreduce_sum_(t: torch.Tensor):
    """In-place sum over the replicas (the small partial-sum buffers of the whole-batch losses)."""
    if world() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=_GROUP)
    return t


def shard(n_total: int, r: int = None, w: int = None):
    """[start, stop) of rank r's share of n_total samples (equal shards; reference batch_size
    is the GLOBAL batch, modules/argmanager.py:95)."""
    r = rank() if r is None else r
    w = world() if w is None else w
    per = n_total // w
    return r * per, (r + 1) * per


def replica_checksums(flats) -> torch.Tensor:
    """[len(flats), 2] float64: sum and index-weighted sum of each flat parameter buffer (any
    difference between replicas, including a permutation, changes them)."""
    rows = []
    for f in flats:
        d = f.detach().double()
        w = torch.arange(1, d.numel() + 1, device=d.device, dtype=torch.float64) / d.numel()
        rows.append(torch.stack([d.sum(), (d * w).sum()]))
    return torch.stack(rows)


def replicas_identical(flats) -> bool:
    """True when every replica of the group holds bit-for-bit the same checksums (collective: every
    rank of the group must call it).  A corrupted all-reduce or a diverged replica shows here."""
    c = replica_checksums(flats)
    if world() == 1:
        return True
    if dist.get_backend(_GROUP) == "gloo":  # gloo gathers host tensors only
        c = c.cpu()
    got = [torch.empty_like(c) for _ in range(world())]
    dist.all_gather(got, c, group=_GROUP)
    return all(torch.equal(g, got[0]) for g in got)
