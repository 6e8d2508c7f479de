"""Margin of tests/test_gpu_train.py::test_explicit_step_matches_autograd_step: the largest relative
loss difference between the explicit and the autograd step per step index, and the parameter
difference statistics (test infrastructure: imports the test's own helpers)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "ducosy-gan_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402

import test_gpu_train as T  # noqa: E402
from oracle import prng  # noqa: E402


def main():
    from modules import trainer
    n, hw, nb, cin, seed = 2, 64, 1, 3, 611
    seeds = prng.step_model_seeds(seed)
    res = {}
    for mode in (False, True):
        trainer._EXPLICIT_STEP = mode
        s = T._system(cin, nb, seeds)
        outs = []
        for i in range(2):
            rA = torch.from_numpy(prng.uniform(seed, f"A{i}", (n, 1, hw, hw), -1, 1)).to("cuda")
            rB = torch.from_numpy(prng.uniform(seed, f"B{i}", (n, 1, hw, hw), -1, 1)).to("cuda")
            mk = torch.from_numpy(prng.bernoulli(seed, f"M{i}", (n, cin - 1, hw, hw), 0.3)).to("cuda")
            outs.append({k: float(v) for k, v in s.train_step(rA, rB, mk).items()})
        params = {f"{t}.{k}": p.detach().clone() for t, m in zip(("GA", "GB", "DA", "DB"), s.models)
                  for k, p in m.named_parameters()}
        res[mode] = (outs, params)
    (oa, pa), (oe, pe) = res[False], res[True]
    for i in range(2):
        worst = max(((abs(oe[i][k] - oa[i][k]) / max(abs(oa[i][k]), 1e-2), k) for k in oa[i]))
        print(f"step {i}: worst relative loss difference {worst[0]:.3e} ({worst[1]})")
    flips = sum(int(((pe[k] - pa[k]).abs() > 1e-6).sum()) for k in pa)
    tot = sum(pa[k].numel() for k in pa)
    print(f"parameters differing by > 1e-6: {flips} of {tot}")
    per = sorted(((int(((pe[k] - pa[k]).abs() > 1e-6).sum()), pa[k].numel(), k) for k in pa), reverse=True)[:12]
    for c, nn, k in per:
        if c:
            print(f"  {k}: {c} of {nn}")


if __name__ == "__main__":
    main()
