"""Guard bands around every output and workspace of the training step (out-of-range store check).

Every tensor the product code allocates through torch.empty / empty_like / zeros / zeros_like /
ones on the device (kernel outputs, padded dgrad buffers, split-K partial slabs, the per-stream
workspaces) is carved out of a larger buffer whose 4 KiB on either side is filled with a canary
byte.  Two steps of the two CycleGANs of config 5 (serial schedule) run with every allocation guarded
(the second replays the recorded weight packs as the batched pack launches),
in the f16x3, f16 and bf16x6 operand modes;
afterwards every guard band must still hold the canary: no kernel stores outside the extent its
host code allocated for it (the two-stream audit).
"""
import math

import pytest
import torch

from oracle import prng
from test_gpu_concurrent import _batch
from test_gpu_train import _system

pytestmark = pytest.mark.gpu
DEV = "cuda"
GUARD = 4096
CANARY = 0x5A


class _Guarded:
    NAMES = ("empty", "empty_like", "zeros", "zeros_like", "ones")

    def __init__(self):
        self.real = {n: getattr(torch, n) for n in self.NAMES}
        self.bufs = []

    def _alloc(self, shape, dtype, device, fill):
        dtype = dtype or torch.get_default_dtype()
        nbytes = math.prod(shape) * torch.empty((), dtype=dtype).element_size()
        base = self.real["empty"](nbytes + 2 * GUARD, dtype=torch.uint8, device=device)
        base.fill_(CANARY)
        t = base[GUARD:GUARD + nbytes].view(dtype).view(tuple(shape))
        if fill is not None:
            t.fill_(fill)
        self.bufs.append((base, nbytes))
        return t

    @staticmethod
    def _shape(size):
        if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)):
            return tuple(size[0])
        return tuple(size)

    def _wrap(self, name, fill):
        real = self.real[name]

        def fn(*size, dtype=None, device=None, **kw):
            if device is None or torch.device(device).type != "cuda" or kw.get("memory_format") not in (
                    None, torch.contiguous_format):
                return real(*size, dtype=dtype, device=device, **kw)
            return self._alloc(self._shape(size), dtype, device, fill)
        return fn

    def _wrap_like(self, name, fill):
        real = self.real[name]

        def fn(x, dtype=None, device=None, **kw):
            dev = device if device is not None else x.device
            if torch.device(dev).type != "cuda" or kw.get("memory_format") not in (None, torch.contiguous_format) \
                    or not x.is_contiguous():
                return real(x, dtype=dtype, device=device, **kw)
            return self._alloc(tuple(x.shape), dtype or x.dtype, dev, fill)
        return fn

    def __enter__(self):
        torch.empty = self._wrap("empty", None)
        torch.zeros = self._wrap("zeros", 0)
        torch.ones = self._wrap("ones", 1)
        torch.empty_like = self._wrap_like("empty_like", None)
        torch.zeros_like = self._wrap_like("zeros_like", 0)
        return self

    def __exit__(self, *exc):
        for n, f in self.real.items():
            setattr(torch, n, f)

    def violations(self):
        torch.cuda.synchronize()
        bad = []
        for base, nbytes in self.bufs:
            head, tail = base[:GUARD], base[GUARD + nbytes:]
            if not (bool((head == CANARY).all()) and bool((tail == CANARY).all())):
                bad.append(nbytes)
        return bad


@pytest.mark.parametrize("mode", ["f16x3", "f16", "bf16x6"])
def test_no_store_outside_allocations(mode):
    from modules.hip import ops
    from modules.trainer import ConcurrentCycleGANs
    n, hw, nb = 2, 64, 2
    cfg = [(3, 821), (2, 822)]
    prev = ops.get_mma()
    ops.set_mma(mode)
    saved_ws = dict(ops._WS)
    try:
        run = ConcurrentCycleGANs([_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg], DEV)
        batches = [_batch(s, 0, n, hw, c) for c, s in cfg]
        torch.cuda.synchronize()
        ops._WS.clear()  # workspaces are re-created (guarded) inside the step
        with _Guarded() as g:
            # two steps: the first allocates the packs and workspaces (guarded) and records the pack
            # plans; the second replays them as the batched pack launches (ops.prepack)
            run.train_step(batches)
            run.train_step(batches)
            torch.cuda.synchronize()
        assert len(g.bufs) > 100, len(g.bufs)
        assert g.violations() == []
    finally:
        ops._WS.clear()
        ops._WS.update(saved_ws)
        ops.set_mma(prev)
