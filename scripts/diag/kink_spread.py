"""Kink spread of the golden Generator fixtures (CPU only): the oracle's input gradient against the
reference's own (tests/golden/gen_*.npz) when every weight is perturbed by a relative 3e-7 (about
the rounding differences of two fp32 implementations).  An element whose ReLU pre-activation sits
within rounding of 0 flips its gradient branch; in a 32 x 32 fixture one flip moves the input
gradient by ~5e-3 relative L2 (measured 5.2e-3 and 1.0e-2 for gen_cin1_nb9_32 in 40 draws; 2.4e-3
for gen_cin3_nb1_64).  tests/test_gpu_models.py sets its input-gradient bar from this."""
import sys, numpy as np, torch
import os
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd")]
from oracle import prng
from oracle import ref_torch as orc
torch.set_num_threads(8)
for fname in ["gen_cin1_nb9_32.npz", "gen_cin3_nb1_64.npz"]:
    z = np.load(os.path.join(ROOT, "tests", "golden", fname))
    cin, nb, cbam, n, hw, seed = [int(v) for v in z["meta"]]
    sd = {k: torch.from_numpy(v) for k, v in prng.init_state_dict(orc.generator_param_shapes(cin, nb, bool(cbam)), seed).items()}
    errs = []
    for t in range(40):
        g = torch.Generator().manual_seed(t)
        p = {k: v * (1 + 3e-7 * torch.randn(v.shape, generator=g)) for k, v in sd.items()}
        x = torch.from_numpy(z["x"]).requires_grad_(True)
        y = orc.generator_forward(p, x, nb, bool(cbam))
        (y * torch.from_numpy(z["R"])).sum().backward()
        r = torch.from_numpy(z["dx"]).double()
        errs.append(float((x.grad.double() - r).norm() / r.norm()))
    print(fname, "dx rel2 under 3e-7 weight perturbations: max %.2e median %.2e" % (max(errs), sorted(errs)[20]), ["%.1e" % e for e in errs])
