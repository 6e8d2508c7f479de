"""Numerical quality of the fp32 HIP path measured against an fp64 run of the oracle.

The north-star bar is 1e-3 relative on generator activations and losses; this test also
records how close the HIP path is to exact arithmetic compared with the reference's own fp32
CPU path (both measured against fp64 on identical weights and inputs).
"""
import numpy as np
import pytest
import torch

from oracle import prng
from oracle import ref_torch as orc

pytestmark = pytest.mark.gpu


def _rel_max(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max())


def _rel_l2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm())


@pytest.mark.parametrize("cin,nb,n,hw", [(3, 2, 2, 64), (1, 9, 1, 32)])
def test_generator_vs_fp64(cin, nb, n, hw):
    from modules.model import Generator
    torch.set_num_threads(8)
    seed = 900 + nb
    sd = {k: torch.from_numpy(v) for k, v in
          prng.init_state_dict(orc.generator_param_shapes(cin, nb, True), seed).items()}
    x = prng.uniform(seed, "x", (n, 1, hw, hw), -1, 1)
    if cin > 1:
        x = np.concatenate([x, prng.bernoulli(seed, "m", (n, cin - 1, hw, hw), 0.3)], 1)
    R = None
    res = {}
    for dt in (torch.float64, torch.float32):
        p = {k: v.to(dt).requires_grad_(True) for k, v in sd.items()}
        xt = torch.from_numpy(x).to(dt).requires_grad_(True)
        y = orc.generator_forward(p, xt, nb, True)
        if R is None:
            R = torch.from_numpy(prng.normal(seed, "R", tuple(y.shape)))
        (y * R.to(dt)).sum().backward()
        res[dt] = (y, xt.grad, {k: v.grad for k, v in p.items()})
    G = Generator(cin, nb).cuda()
    G.load_state_dict(sd)
    xg = torch.from_numpy(x).cuda().requires_grad_(True)
    y = G(xg)
    (y * R.cuda()).sum().backward()
    y64, dx64, g64 = res[torch.float64]
    y32, dx32, g32 = res[torch.float32]
    e_hip, e_cpu = _rel_max(y, y64), _rel_max(y32, y64)
    print(f"\n[G cin{cin} nb{nb} {hw}x{hw}] out max-rel vs fp64: hip {e_hip:.2e}  cpu-fp32 {e_cpu:.2e}")
    print(f"  dx rel-L2 vs fp64: hip {_rel_l2(xg.grad, dx64):.2e}  cpu-fp32 {_rel_l2(dx32, dx64):.2e}")
    worst = max((_rel_l2(pp.grad, g64[k]), k) for k, pp in G.named_parameters() if pp.dim() == 4)
    print(f"  worst weight-grad rel-L2 vs fp64: hip {worst[0]:.2e} ({worst[1]})")
    assert e_hip < 1e-4  # activations: 10x inside the 1e-3 bar
    assert _rel_l2(xg.grad, dx64) < 1e-2
    assert worst[0] < 1e-2
