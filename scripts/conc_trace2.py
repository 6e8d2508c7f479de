"""Find the first op whose output differs between the sequential run and the overlapping
two-stream schedule (tests/test_gpu_concurrent.py setting): every public function of
modules.hip.ops and every ConvGeom method is wrapped to record an integer checksum of each
tensor it returns (on the current stream, no host sync).  Host issue order is the same in
both runs, so the two records align op by op.   python scripts/conc_trace2.py MODE ATTEMPTS"""
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_train import _system
from test_gpu_concurrent import _batch
from modules.hip import ops

n, hw, nb, steps = 2, 64, 2, 3
cfg = [(3, 801), (2, 802)]
ops.set_mma(sys.argv[1])
attempts = int(sys.argv[2])
REC = []


def cks(t):
    if t.dtype in (torch.float32, torch.int32):
        return t.contiguous().view(torch.int32).to(torch.int64).sum()
    if t.dtype == torch.float64:
        return t.contiguous().view(torch.int64).sum()
    return t.float().sum()


def walk(x, out):
    if torch.is_tensor(x):
        out.append(cks(x))
    elif isinstance(x, (tuple, list)):
        for y in x:
            walk(y, out)
    elif isinstance(x, ops.INStats):
        for y in (x.scale, x.shift, x.xmax, x.xargmax):
            if y is not None:
                out.append(cks(y))


def desc(a):
    if torch.is_tensor(a):
        return f"T{tuple(a.shape)}"
    if isinstance(a, ops.ConvGeom):
        return f"Geom({a.cin}->{a.cout},k{a.k},s{a.stride},up{a.up},pads{a.pads},mode{a.pad_mode})"
    if isinstance(a, ops.Src):
        return f"Src({a.N},{a.H},{a.W},{a.C},nchw={a.strides[1] != 1})"
    return type(a).__name__


SAVE = {}


def wrap(name, fn):
    def w(*a, **k):
        if name == "ConvGeom.forward" and isinstance(a[0], ops.ConvGeom) and a[0].cout == 1 and a[0].cin == 512:
            pre = [x.t.clone() for x in a if isinstance(x, ops.Src)] + [x.clone() for x in a if torch.is_tensor(x)]
            pro = k.get("pro")
            pre += [pro[0].clone(), pro[1].clone()] if pro else []
            pre += [k["bias"].clone()] if k.get("bias") is not None else []
        r = fn(*a, **k)
        if name == "ConvGeom.forward" and isinstance(a[0], ops.ConvGeom) and a[0].cout == 1 and a[0].cin == 512:
            SAVE[len(REC)] = pre + [r.clone()]
        cs = []
        walk(r, cs)
        REC.append((name + " " + " ".join(desc(x) for x in a) + (" pro" if k.get("pro") else "")
                    + (" bias" if k.get("bias") is not None else ""), cs))
        return r
    return w


import os  # noqa: E402
ONLY = os.environ.get("TRACE_ONLY", "")  # "conv": ConvGeom passes only (fewer extra kernels)
if ONLY != "conv":
    for name in dir(ops):
        f = getattr(ops, name)
        if callable(f) and not name.startswith("_") and getattr(f, "__module__", "") == ops.__name__ \
                and not isinstance(f, type) and name not in ("workspace", "set_mma", "get_mma"):
            setattr(ops, name, wrap(name, f))
for m in ("forward", "forward_in_stats", "dgrad", "wgrad", "pack_fwd", "pack_dgrad"):
    setattr(ops.ConvGeom, m, wrap("ConvGeom." + m, getattr(ops.ConvGeom, m)))


def run(overlap):
    REC.clear()
    SAVE.clear()
    systems = [_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg]
    streams = [torch.cuda.Stream() for _ in cfg]
    cur = torch.cuda.current_stream()
    for i in range(steps):
        for sysm, st, (c, s) in zip(systems, streams, cfg):
            b = _batch(s, i, n, hw, c)
            if not overlap:
                sysm.train_step(*b)
                continue
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                for t in b:
                    t.record_stream(st)
                sysm.train_step(*b)
        for st in streams:
            cur.wait_stream(st)
        torch.cuda.synchronize()
    return [(nm, [int(c) for c in cs]) for nm, cs in REC], dict(SAVE)


want, wsave = run(False)
print("ops recorded:", len(want), flush=True)
for a in range(attempts):
    got, gsave = run(True)
    assert [x[0] for x in got] == [x[0] for x in want]
    if a == 0:
        print("op 130-136:", [want[j][0] for j in range(130, 137)], flush=True)
    diffs = [i for i, (g, w) in enumerate(zip(got, want)) if g[1] != w[1]]
    if diffs:
        i0 = diffs[0]
        print(f"attempt {a}: {len(diffs)} ops differ; first at op {i0}: {want[i0][0]}", flush=True)
        for i in diffs[:8]:
            print("   ", i, want[i][0], [int(x != y) for x, y in zip(want[i][1], got[i][1])])
        if i0 in wsave:
            names = ["src", "wpack", "scale", "shift", "bias", "out"]
            for nm_, x, y in zip(names, wsave[i0], gsave[i0]):
                d = (x - y).abs()
                print(f"    {nm_} {tuple(x.shape)}: {int((d > 0).sum())} differ, max {float(d.max()):.3g} "
                      f"(|ref| max {float(x.abs().max()):.3g})", flush=True)
            o1, o2 = wsave[i0][-1].flatten(), gsave[i0][-1].flatten()
            idx = (o1 != o2).nonzero().flatten()[:8]
            print("    out idx", idx.tolist(), "ref", o1[idx].tolist(), "got", o2[idx].tolist())
    else:
        print(f"attempt {a}: identical", flush=True)
