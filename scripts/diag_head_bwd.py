"""Diagnose the fused head dgrad + IN backward against float64 at one size (where the error sits)."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "ducosy-gan_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import prng  # noqa: E402
from modules.hip import ops  # noqa: E402
from modules.hip.lib import ACT_RELU, DCS_PAD_REFLECT  # noqa: E402

DEV = "cuda"


def rnd(shape, seed, name, lo=-1.0, hi=1.0):
    return torch.from_numpy(prng.uniform(seed, name, shape, lo, hi))


N, H, W = [int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (2, 512, 512))]
ops.set_mma("f16x3")
g = ops.ConvGeom(64, 1, 7, 1, (3, 3, 3, 3), DCS_PAD_REFLECT)
y = (rnd((N, 64, H, W), 51, "y") * 3.0 + 0.5).float().to(DEV).permute(0, 2, 3, 1).contiguous()
w = torch.from_numpy(prng.normal(52, "w", (1, 64, 7, 7), 0, 0.05)).float().to(DEV)
dout = (rnd((N, 1, H, W), 53, "dy") * 1e-3).float().to(DEV)
st = ops.in_stats(y, want_max=True)
yd = y.double().cpu().permute(0, 3, 1, 2).clone().requires_grad_(True)
m = yd.mean((2, 3), keepdim=True)
v = yd.var((2, 3), unbiased=False, keepdim=True)
rstd = 1.0 / torch.sqrt(v + 1e-5)
print("scale rel err", float(((st.scale.double().cpu() - rstd[:, :, 0, 0]).abs() / rstd[:, :, 0, 0]).max()))
print("shift abs err", float((st.shift.double().cpu() + (m * rstd)[:, :, 0, 0]).abs().max()))
a = torch.relu((yd - m) * rstd)
out = F.conv2d(F.pad(a, (3, 3, 3, 3), mode="reflect"), w.double().cpu())
out.backward(dout.double().cpu())
ref = yd.grad.permute(0, 2, 3, 1)
wk = g.pack_dgrad(w)
dyn = dout.permute(0, 2, 3, 1).contiguous()
fused = ops.head_dgrad_in(dyn, wk, y, st, ACT_RELU).double().cpu()
da = g.dgrad(dyn, wk, H, W)
sep = ops.in_act_backward(da, y, st, ACT_RELU).double().cpu()
# da against float64 (the conv adjoint alone)
ad = a.detach().clone().requires_grad_(True)
o2 = F.conv2d(F.pad(ad, (3, 3, 3, 3), mode="reflect"), w.double().cpu())
o2.backward(dout.double().cpu())
da_ref = ad.grad.permute(0, 2, 3, 1)
print("da relmax", float((da.double().cpu() - da_ref).abs().max() / da_ref.abs().max()))
for name, t in (("fused", fused), ("separate", sep)):
    d = (t - ref).abs()
    i = int(d.argmax())
    idx = [int(q) for q in torch.unravel_index(torch.tensor(i), d.shape)]
    print(name, "relmax", float(d.max() / ref.abs().max()), "at", idx, "got", float(t.flatten()[i]), "ref",
          float(ref.flatten()[i]), "max|ref|", float(ref.abs().max()))
    print(name, "rel L2", float(d.norm() / ref.norm()))
