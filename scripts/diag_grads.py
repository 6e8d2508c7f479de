"""Step-0 gradients of the explicit and the autograd step (tests/test_gpu_train.py's setup): relative
L2 difference per parameter, worst first (test infrastructure: imports the test's own helpers)."""
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
    from modules.optim import FusedAdam
    n, hw, nb, cin, seed = 2, 64, 1, 3, 611
    seeds = prng.step_model_seeds(seed)
    grads = {}
    orig = FusedAdam.step
    from modules.hip import ops
    for mode in ((False, True), (True, True), (False, False), (True, False)):
        trainer._EXPLICIT_STEP = mode[0]
        ops._SUBWIN = mode[1]
        s = T._system(cin, nb, seeds)
        cap = []

        def step(self, closure=None, cap=cap):
            cap.append({id(p): p.grad.detach().clone() for p in self.param_groups[0]["params"]})
            return orig(self, closure)
        FusedAdam.step = step
        names = {id(p): f"{t}.{k}" for t, m in zip(("GA", "GB", "DA", "DB"), s.models) for k, p in m.named_parameters()}
        per_step = []
        for i in range(2):
            cap.clear()
            rA = torch.from_numpy(prng.uniform(seed, f"A{i}", (n, 1, hw, hw), -1, 1)).to("cuda")
            rB = torch.from_numpy(prng.uniform(seed, f"B{i}", (n, 1, hw, hw), -1, 1)).to("cuda")
            mk = torch.from_numpy(prng.bernoulli(seed, f"M{i}", (n, cin - 1, hw, hw), 0.3)).to("cuda")
            s.train_step(rA, rB, mk)
            g = {}
            for c in cap:
                for pid, v in c.items():
                    g[names[pid]] = v
            params = {f"{t}.{k}": p.detach().clone() for t, m in zip(("GA", "GB", "DA", "DB"), s.models)
                      for k, p in m.named_parameters()}
            per_step.append((g, params))
        FusedAdam.step = orig
        grads[mode] = per_step
    tag = {(False, True): "A1", (True, True): "E1", (False, False): "A0", (True, False): "E0"}
    for x, y in (((False, True), (True, True)), ((False, False), (True, False)), ((True, False), (True, True)),
                 ((False, False), (False, True))):
      print(f"== {tag[x]} vs {tag[y]}")
      for i in range(2):
        (ga, pa), (ge, pe) = grads[x][i], grads[y][i]
        flips = sum(int(((pe[k] - pa[k]).abs() > 1e-6).sum()) for k in pa)
        print(f"step {i}: parameters differing by > 1e-6 after it: {flips}")
        rows = []
        for k in ga:
            a, e = ga[k].double(), ge[k].double()
            rows.append((float((a - e).norm() / max(float(a.norm()), 1e-30)), float((a - e).abs().max()), k))
        rows.sort(reverse=True)
        for r, m, k in rows[:3]:
            print(f"  {k:40s} grad rel L2 {r:.3e}  max abs {m:.3e}")


if __name__ == "__main__":
    main()
