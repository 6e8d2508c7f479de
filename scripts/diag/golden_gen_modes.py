"""Golden-fixture Generator (tests/golden/*.npz): output and gradient errors per MFMA operand mode."""
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

for fname in sys.argv[1:] or ["gen_cin1_nb9_32.npz"]:
    z = np.load(os.path.join(ROOT, "tests", "golden", fname))
    cin, nb, cbam, n, hw, seed = [int(v) for v in z["meta"]]
    sd = {k: torch.from_numpy(v) for k, v in prng.init_state_dict(orc.generator_param_shapes(cin, nb, bool(cbam)), seed).items()}
    for mode in ("f32", "bf16x6", "f16x3"):
        ops.set_mma(mode)
        G = Generator(input_channels=cin, num_residual_blocks=nb, use_cbam=bool(cbam))
        G.load_state_dict(sd)
        G = G.cuda()
        x = torch.from_numpy(z["x"]).cuda().requires_grad_(True)
        y = G(x)
        fy = float((y.detach().double().cpu() - torch.from_numpy(z["y"]).double()).abs().max() / np.abs(z["y"]).max())
        (y * torch.from_numpy(z["R"]).cuda()).sum().backward()
        r = torch.from_numpy(z["dx"]).double()
        fdx = float((x.grad.double().cpu() - r).norm() / r.norm())
        gw = {}
        for name, p in G.named_parameters():
            if name.endswith(".bias"):
                continue
            gn = float(z[f"gnorm:{name}"])
            gw[name] = abs(float(p.grad.double().norm()) - gn) / gn
        worst = sorted(gw.items(), key=lambda kv: -kv[1])[:3]
        print(fname, mode, "y", f"{fy:.2e}", "dx", f"{fdx:.2e}", "worst |gnorm| rel", [(k, f"{v:.1e}") for k, v in worst], flush=True)
