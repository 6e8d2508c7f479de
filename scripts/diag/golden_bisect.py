"""Bisect a golden-fixture Generator backward discrepancy: the gradient reaching the last residual
block's CBAM (dL/d block output) and the one leaving it, HIP vs the oracle, per operand mode."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import prng  # noqa: E402
from oracle import ref_torch as orc  # noqa: E402
from modules.hip import ops  # noqa: E402
from modules.model import Generator  # noqa: E402

fname = sys.argv[1] if len(sys.argv) > 1 else "gen_cin3_nb1_64.npz"
z = np.load(os.path.join(ROOT, "tests", "golden", fname))
cin, nb, cbam, n, hw, seed = [int(v) for v in z["meta"]]
sd = {k: torch.from_numpy(v) for k, v in prng.init_state_dict(orc.generator_param_shapes(cin, nb, bool(cbam)), seed).items()}
# oracle with retained intermediates
p = {k: v.clone().double().requires_grad_(True) for k, v in sd.items()}
x = torch.from_numpy(z["x"]).double().requires_grad_(True)
keep = {}
h = F.conv2d(F.pad(x, (3, 3, 3, 3), mode="reflect"), p["model.1.weight"], p["model.1.bias"])
h = F.relu(orc._inorm(h))
for idx in (4, 7):
    h = F.relu(orc._inorm(F.conv2d(h, p[f"model.{idx}.weight"], p[f"model.{idx}.bias"], stride=2, padding=1)))
for b in range(nb):
    h.retain_grad(); keep[f"in{b}"] = h
    h = orc.residual_block(p, f"model.{10 + b}", h, bool(cbam))
h.retain_grad(); keep["out_res"] = h
u = 10 + nb
for idx in (u + 1, u + 5):
    h = F.interpolate(h, scale_factor=2, mode="nearest")
    h = F.relu(orc._inorm(F.conv2d(h, p[f"model.{idx}.weight"], p[f"model.{idx}.bias"], padding=1)))
y = torch.tanh(F.conv2d(F.pad(h, (3, 3, 3, 3), mode="reflect"), p[f"model.{u + 9}.weight"], p[f"model.{u + 9}.bias"]))
(y * torch.from_numpy(z["R"]).double()).sum().backward()

rec = {}
orig_cb = ops.cbam_backward
orig_dg = ops.ConvGeom.dgrad


def cb_hook(dout, *a, **k):
    rec.setdefault("cb_dout", []).append(dout.clone())
    r = orig_cb(dout, *a, **k)
    rec.setdefault("cb_dy", []).append(r[0].clone())
    return r


def dg_hook(self, dy, *a, **k):
    out = orig_dg(self, dy, *a, **k)
    rec.setdefault("dgrad", []).append((self, out.clone()))
    return out


ops.cbam_backward = cb_hook
ops.ConvGeom.dgrad = dg_hook
import modules.hip.networks as net  # noqa: E402
net.ops.cbam_backward = cb_hook
rel2 = lambda a, b: float((a.double().cpu() - b.double()).norm() / b.double().norm())
for mode in ("f32", "bf16x6", "f16x3"):
    rec.clear()
    ops.set_mma(mode)
    G = Generator(input_channels=cin, num_residual_blocks=nb, use_cbam=bool(cbam))
    G.load_state_dict(sd)
    G = G.cuda()
    xd = torch.from_numpy(z["x"]).cuda().requires_grad_(True)
    (G(xd) * torch.from_numpy(z["R"]).cuda()).sum().backward()
    last = nb - 1
    dout = rec["cb_dout"][0].permute(0, 3, 1, 2)  # first CBAM backward = last block
    line = [f"dout(block {last})={rel2(dout, keep['out_res'].grad):.2e}"]
    res = [o for g, o in rec["dgrad"] if g.cin == 256 and g.cout == 256 and g.k == 3 and g.stride == 1 and g.up == 1]
    for b in range(nb):
        line.append(f"d in{b}={rel2(res[2 * (nb - 1 - b) + 1].permute(0, 3, 1, 2), keep[f'in{b}'].grad):.2e}")
    line.append(f"dx={rel2(xd.grad, x.grad):.2e}")
    print(fname, mode, " ".join(line), flush=True)
