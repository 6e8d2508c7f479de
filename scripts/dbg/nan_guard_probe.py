"""Run train steps with every device allocation NaN-filled and padded by NaN guard regions
(scripts/dbg/guard_alloc.cpp), checking the outputs of every modules.hip.ops function and
ConvGeom method for NaN: the first op that produces NaN read memory outside its tensors or
memory no kernel wrote.   python scripts/dbg/nan_guard_probe.py MODE"""
import os
import sys
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
alloc = torch.cuda.memory.CUDAPluggableAllocator(os.path.join(HERE, "libguard_alloc.so"), "guard_alloc", "guard_free")
torch.cuda.memory.change_current_allocator(alloc)

ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
for p in ("tests", "ducosy-gan_amd", ""):
    sys.path.insert(0, os.path.join(ROOT, p))
from oracle import prng  # noqa: E402
from test_gpu_train import _system  # noqa: E402
from test_gpu_concurrent import _batch  # noqa: E402
from modules.hip import ops  # noqa: E402

ops.set_mma(sys.argv[1])
n, hw, nb, steps = 2, 64, 2, 2
cfg = [(3, 801), (2, 802)]
found = []


def has_nan(x):
    if torch.is_tensor(x):
        return x.is_floating_point() and bool(torch.isnan(x).any())
    if isinstance(x, (tuple, list)):
        return any(has_nan(y) for y in x)
    if isinstance(x, ops.INStats):
        return any(has_nan(y) for y in (x.scale, x.shift, x.xmax) if y is not None)
    return False


def desc(a):
    if torch.is_tensor(a):
        return f"T{tuple(a.shape)}"
    if isinstance(a, ops.ConvGeom):
        return f"Geom(cin={a.cin},cout={a.cout},k={a.k},s={a.stride},up={a.up},pads={a.pads})"
    if isinstance(a, ops.Src):
        return f"Src({a.N},{a.H},{a.W},{a.C})"
    return type(a).__name__


def wrap(name, fn):
    def w(*a, **k):
        bad_in = has_nan([x for x in a if torch.is_tensor(x)])
        r = fn(*a, **k)
        if not found and not bad_in and has_nan(r):
            found.append(name)
            print("FIRST NaN output:", name, [desc(x) for x in a], {kk: desc(v) for kk, v in k.items()}, flush=True)
        return r
    return w


for name in dir(ops):
    f = getattr(ops, name)
    if callable(f) and not name.startswith("_") and getattr(f, "__module__", "") == ops.__name__ \
            and not isinstance(f, type) and name not in ("workspace", "set_mma", "get_mma"):
        setattr(ops, name, wrap(name, f))
for m in ("forward", "forward_in_stats", "dgrad", "wgrad", "pack_fwd", "pack_dgrad"):
    setattr(ops.ConvGeom, m, wrap("ConvGeom." + m, getattr(ops.ConvGeom, m)))

import gc  # noqa: E402
for c, s in cfg:
    m = _system(c, nb, prng.step_model_seeds(s))
    for i in range(steps):
        out = {k: float(v) for k, v in m.train_step(*_batch(s, i, n, hw, c)).items()}
        print(f"cin {c} step {i}:", {k: round(v, 5) for k, v in list(out.items())[:4]}, flush=True)
    del m, out
    ops._WS.clear()  # free the scratch buffers too: every block's guards are checked at free
    gc.collect()
    torch.cuda.synchronize()
print("NaN-producing op:", found[0] if found else "none")
print("done (guard reports, if any, are on stderr)")
