"""Per-step loss deviation of the HIP train step from the golden reference fixture (diagnostic).
    python scripts/step_drift.py            (uses DUCOSY_HIP_LIB if set)"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import prng  # noqa: E402
from test_gpu_train import _system  # noqa: E402

z = np.load(os.path.join(ROOT, "tests", "golden", "steps_64.npz"))
n, hw, nb, cin, steps, seed = [int(v) for v in z["meta"]]
s = _system(cin, nb, prng.step_model_seeds(seed))
for i in range(steps):
    rA = torch.from_numpy(prng.uniform(seed, f"A{i}", (n, 1, hw, hw), -1, 1)).cuda()
    rB = torch.from_numpy(prng.uniform(seed, f"B{i}", (n, 1, hw, hw), -1, 1)).cuda()
    mk = torch.from_numpy(prng.bernoulli(seed, f"M{i}", (n, cin - 1, hw, hw), 0.3)).cuda()
    out = {k: float(v) for k, v in s.train_step(rA, rB, mk).items()}
    print(i, "  ".join(f"{k[5:]}:{(v - float(z[k][i])) / float(z[k][i]):+.1e}" for k, v in out.items()))
