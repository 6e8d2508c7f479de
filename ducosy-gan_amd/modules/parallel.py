"""Data parallelism: one process per GPU, torch.distributed over RCCL (backend "nccl").

Replaces the reference's single-process nn.DataParallel (modules/trainer.py:333-338), which
scatters every G/D call over 8 GPUs, re-broadcasts all parameters per call and reduces
gradients to cuda:0.  Here each rank owns full replicas of G_A2B, G_B2A, D_A, D_B and its own
batch shard; per optimizer step there is exactly ONE all-reduce of that optimizer's flat
gradient buffer (FusedAdam.flat_g: 91.6 MB for the G pair, 11.05 MB per D at cin 3), averaged
over ranks.  Initial weights are broadcast from rank 0 once.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


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


def local_device_index() -> int:
    """GPU of this process: LOCAL_RANK (one process per GPU).  DUCOSY_DEVICE_OVERRIDE pins
    every rank to one device — for rehearsing the multi-process path on a single GPU with
    DUCOSY_DIST_BACKEND=gloo (RCCL does not allow two ranks on one device)."""
    o = os.environ.get("DUCOSY_DEVICE_OVERRIDE")
    return int(o) if o not in (None, "") else int(os.environ.get("LOCAL_RANK", "0"))


def broadcast_(flat: torch.Tensor, src: int = 0):
    if world() > 1:
        dist.broadcast(flat, src)
    return flat


def allreduce_mean_(flat: torch.Tensor):
    """In-place mean over ranks of a flat gradient buffer (one collective)."""
    w = world()
    if w == 1:
        return flat
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    if flat.is_cuda:
        from .hip import ops
        ops.scale_add_(flat, flat, 1.0 / w - 1.0)  # flat *= 1/w on the device kernel
    else:
        flat.mul_(1.0 / w)
    return flat


def allreduce_sum_(t: torch.Tensor):
    """In-place sum over ranks (the small partial-sum buffers of the global-statistics losses)."""
    if world() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def shard(n_total: int, r: int = None, w: int = None):
    """[start, stop) of rank r's share of n_total samples (equal shards; reference batch_size
    is the GLOBAL batch, modules/argmanager.py:95)."""
    r = rank() if r is None else r
    w = world() if w is None else w
    per = n_total // w
    return r * per, (r + 1) * per
