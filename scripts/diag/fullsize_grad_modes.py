"""Config-2 gradient errors (relative L2 vs the oracle) per parameter, per MFMA operand mode."""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from oracle import prng  # noqa: E402
from oracle import ref_torch as orc  # noqa: E402

torch.set_num_threads(16)
HW, NB, CIN, n, seed = 512, 9, 3, 2, 911
sd = {k: torch.from_numpy(v) for k, v in prng.init_state_dict(orc.generator_param_shapes(CIN, NB, True), seed).items()}
x = torch.from_numpy(prng.uniform(seed, "A0", (n, 1, HW, HW), -1, 1))
m = torch.from_numpy(prng.bernoulli(seed, "M0", (n, CIN - 1, HW, HW), 0.3))
dout = torch.from_numpy(prng.normal(seed, "dout", (n, 1, HW, HW), 0, 1e-3))
pr = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
xr = x.clone().requires_grad_(True)
(orc.generator_forward(pr, torch.cat([xr, m], 1), NB, True) * dout).sum().backward()
from modules.hip import ops  # noqa: E402
from modules.model import Generator  # noqa: E402
out = {}
for mode in sys.argv[1:] or ["f32", "bf16x6", "f16x3"]:
    ops.set_mma(mode)
    G = Generator(input_channels=CIN, num_residual_blocks=NB, use_cbam=True)
    G.load_state_dict(sd)
    G.cuda()
    xd = x.cuda().requires_grad_(True)
    G(xd, m.cuda()).backward(dout.cuda())
    names = dict(G.named_parameters())
    e = {}
    for k, v in pr.items():
        if v.dim() == 1 and k != f"model.{10 + NB + 9}.bias":
            continue
        g = names[k].grad.cpu().double()
        r = v.grad.double()
        e[k] = float((g - r).norm() / r.norm())
    e["dx"] = float((xd.grad.cpu().double() - xr.grad.double()).norm() / xr.grad.double().norm())
    out[mode] = e
    worst = sorted(e.items(), key=lambda kv: -kv[1])[:6]
    print(mode, [(k, round(v, 5)) for k, v in worst], flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "fullsize_grad_modes.json"), "w"), indent=1)
