"""Hunt an intra-kernel race: record every modules.hip.ops call (and ConvGeom method) of one
train step, then replay each call repeatedly while a second stream runs heavy unrelated work
(the residual-geometry bf16x6 weight gradient in a loop) and compare every replay's outputs bit
for bit with a quiet replay.   python scripts/race_hunt.py MODE REPS"""
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_train import _system
from test_gpu_concurrent import _batch
from modules.hip import ops
from modules.hip.lib import DCS_PAD_REFLECT

ops.set_mma(sys.argv[1])
reps = int(sys.argv[2])
CALLS = []
ORIG = {}


def wrap(name, fn):
    def w(*a, **k):
        r = fn(*a, **k)
        if not name.endswith("_"):
            CALLS.append((name, fn, a, k))
        return r
    return w


for name in dir(ops):
    f = getattr(ops, name)
    if callable(f) and not name.startswith("_") and getattr(f, "__module__", "") == ops.__name__ \
            and not isinstance(f, type) and name not in ("workspace", "set_mma", "get_mma"):
        setattr(ops, name, wrap(name, f))
for m in ("forward", "forward_in_stats", "dgrad", "wgrad", "pack_fwd", "pack_dgrad"):
    setattr(ops.ConvGeom, m, wrap("ConvGeom." + m, getattr(ops.ConvGeom, m)))

n, hw, nb = 2, 64, 2
sysm = _system(2, nb, prng.step_model_seeds(802))
sysm.train_step(*_batch(802, 0, n, hw, 2))
torch.cuda.synchronize()
calls = list(CALLS)
print("recorded calls:", len(calls), flush=True)


def flat(x, out):
    if torch.is_tensor(x):
        out.append(x)
    elif isinstance(x, (tuple, list)):
        for y in x:
            flat(y, out)
    elif isinstance(x, ops.INStats):
        for y in (x.scale, x.shift, x.xmax, x.xargmax):
            if y is not None:
                out.append(y)
    return out


g = ops.ConvGeom(256, 256, 3, 1, (1, 1, 1, 1), DCS_PAD_REFLECT)
xn = torch.randn(8, 64, 64, 256, device="cuda")
sn, sa = torch.cuda.Stream(), torch.cuda.Stream()
bad = {}
seen = set()
for idx, (name, fn, a, k) in enumerate(calls):
    sig = (name, tuple(tuple(t.shape) for t in a if torch.is_tensor(t)))
    if sig in seen:
        continue
    seen.add(sig)
    ref = [t.clone() for t in flat(fn(*a, **k), [])]
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream()
    sn.wait_stream(cur)
    sa.wait_stream(cur)
    with torch.cuda.stream(sn):
        for _ in range(reps * 3):
            g.wgrad(xn, ops.Src.nhwc(xn))
    outs = []
    with torch.cuda.stream(sa):
        for _ in range(reps):
            outs.append(flat(fn(*a, **k), []))
    cur.wait_stream(sn)
    cur.wait_stream(sa)
    torch.cuda.synchronize()
    nbad = sum(any(not torch.equal(x, y) for x, y in zip(o, ref)) for o in outs)
    if nbad:
        bad[sig] = nbad
        print(f"RACE? {name} {sig[1]}: {nbad}/{reps} replays differ", flush=True)
print("distinct calls replayed:", len(seen), "suspects:", len(bad))
