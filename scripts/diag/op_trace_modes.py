"""Record every ops-level call's output in a Generator forward+backward (golden fixture) per MFMA
operand mode and report, op by op, the relative L2 difference of each mode's output to f32's."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import prng  # noqa: E402
from oracle import ref_torch as orc  # noqa: E402
from modules.hip import ops  # noqa: E402
from modules.model import Generator  # noqa: E402

fname = sys.argv[1] if len(sys.argv) > 1 else "gen_cin3_nb1_64.npz"
z = np.load(os.path.join(ROOT, "tests", "golden", fname))
cin, nb, cbam, n, hw, seed = [int(v) for v in z["meta"]]
sd = {k: torch.from_numpy(v) for k, v in prng.init_state_dict(orc.generator_param_shapes(cin, nb, bool(cbam)), seed).items()}
trace = []


def wrap(name, fn, method=False):
    def w(*a, **k):
        out = fn(*a, **k)
        o = out[0] if isinstance(out, tuple) else out
        if isinstance(o, torch.Tensor):
            geo = ""
            if method:
                g = a[0]
                geo = f"[{g.cin}->{g.cout} k{g.k} s{g.stride} u{g.up}]"
            trace.append((name + geo, o.detach().double().cpu().clone()))
        return out
    return w


for nm in ("forward", "forward_in_stats", "dgrad", "wgrad"):
    setattr(ops.ConvGeom, nm, wrap(nm, getattr(ops.ConvGeom, nm), True))
for nm in ("in_apply", "in_act_backward", "act_backward", "cbam_forward", "cbam_backward", "channel_sum", "pack_nhwc4"):
    setattr(ops, nm, wrap(nm, getattr(ops, nm)))
res = {}
for mode in ("f32", "bf16x6", "f16x3"):
    trace.clear()
    ops.set_mma(mode)
    G = Generator(input_channels=cin, num_residual_blocks=nb, use_cbam=bool(cbam))
    G.load_state_dict(sd)
    G = G.cuda()
    xd = torch.from_numpy(z["x"]).cuda().requires_grad_(True)
    (G(xd) * torch.from_numpy(z["R"]).cuda()).sum().backward()
    res[mode] = list(trace)
for mode in ("bf16x6", "f16x3"):
    print("==", fname, mode, "vs f32")
    for (na, a), (nb_, b) in zip(res[mode], res["f32"]):
        d = float((a - b).norm() / max(b.norm(), 1e-30)) if a.shape == b.shape else -1
        flag = "  <<<" if d > 1e-4 else ""
        print(f"  {na:45s} {tuple(a.shape)!s:22s} {d:.2e}{flag}")
