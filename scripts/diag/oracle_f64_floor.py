"""How much of the config-2 gradient error at 512x512 is the fp32 oracle's own rounding: the oracle
(oracle/ref_torch.py) in float32 against the same oracle in float64, per parameter (relative L2),
on the inputs of tests/test_gpu_fullsize.py::test_fullsize_generator_stages_and_grads_vs_oracle.
With --hip MODE... (GPU) the HIP Generator's gradients in each operand mode against float64 too.
Writes gpurun_out/oracle_f64_floor.json."""
import json
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from oracle import prng  # noqa: E402
from oracle import ref_torch as orc  # noqa: E402

torch.set_num_threads(min(16, os.cpu_count() or 1))
HW, NB, CIN, n, seed = 512, 9, 3, 2, 911
sd = {k: torch.from_numpy(v) for k, v in prng.init_state_dict(orc.generator_param_shapes(CIN, NB, True), seed).items()}
x = torch.from_numpy(prng.uniform(seed, "A0", (n, 1, HW, HW), -1, 1))
m = torch.from_numpy(prng.bernoulli(seed, "M0", (n, CIN - 1, HW, HW), 0.3))
dout = torch.from_numpy(prng.normal(seed, "dout", (n, 1, HW, HW), 0, 1e-3))


def oracle_grads(dtype):
    pr = {k: v.to(dtype).clone().requires_grad_(True) for k, v in sd.items()}
    xr = x.to(dtype).clone().requires_grad_(True)
    (orc.generator_forward(pr, torch.cat([xr, m.to(dtype)], 1), NB, True) * dout.to(dtype)).sum().backward()
    g = {k: v.grad.double() for k, v in pr.items() if not (v.dim() == 1 and k != f"model.{10 + NB + 9}.bias")}
    g["dx"] = xr.grad.double()
    return g


def rel(a, b):
    return float((a - b).norm() / b.norm())


t0 = time.time()
g64 = oracle_grads(torch.float64)
g32 = oracle_grads(torch.float32)
out = {"oracle_f32": {k: rel(g32[k], g64[k]) for k in g64}}
print(f"oracle f32 vs f64 ({time.time() - t0:.0f} s): worst",
      sorted(out["oracle_f32"].items(), key=lambda kv: -kv[1])[:6], flush=True)
modes = [a for a in sys.argv[1:] if not a.startswith("-")]
if modes:
    from modules.hip import ops  # noqa: E402
    from modules.model import Generator  # noqa: E402
    for mode in modes:
        ops.set_mma(mode)
        G = Generator(input_channels=CIN, num_residual_blocks=NB, use_cbam=True)
        G.load_state_dict(sd)
        G.cuda()
        xd = x.cuda().requires_grad_(True)
        G(xd, m.cuda()).backward(dout.cuda())
        names = dict(G.named_parameters())
        e = {k: rel(names[k].grad.cpu().double(), g64[k]) for k in g64 if k != "dx"}
        e["dx"] = rel(xd.grad.cpu().double(), g64["dx"])
        out[mode] = e
        print(mode, "vs f64: worst", sorted(e.items(), key=lambda kv: -kv[1])[:6], flush=True)
cb = lambda d: max(v for k, v in d.items() if ".cbam." in k)
other = lambda d: max(v for k, v in d.items() if ".cbam." not in k)
print({k: {"cbam_max": cb(d), "other_max": other(d)} for k, d in out.items()})
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "oracle_f64_floor.json"), "w"), indent=1)
