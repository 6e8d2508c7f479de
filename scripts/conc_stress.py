"""Rate of two-stream divergence at the full-step level: R fresh pairs of CycleGANs (soft
tissue cin 3, lung cin 2) step concurrently on two HIP streams; every loss and parameter is
compared with the same models stepped one after the other.
    python scripts/conc_stress.py MODE R"""
import json
import sys

import torch

sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_concurrent import _batch
from test_gpu_train import _system
from modules.hip import ops
from modules.trainer import ConcurrentCycleGANs

mode, R = sys.argv[1], int(sys.argv[2])
ops.set_mma(mode)
n, hw, nb, steps = 2, 64, 2, 3
cfg = [(3, 801), (2, 802)]
seq = [_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg]
want = [[{k: float(v) for k, v in m.train_step(*_batch(s, i, n, hw, c)).items()} for i in range(steps)]
        for m, (c, s) in zip(seq, cfg)]
wantp = [torch.cat([m.optimizer_G.flat_p, m.optimizer_D_A.flat_p, m.optimizer_D_B.flat_p]) for m in seq]
bad = []
for r in range(R):
    run = ConcurrentCycleGANs([_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg], "cuda", schedule="concurrent")
    got = [[], []]
    for i in range(steps):
        outs = run.train_step([_batch(s, i, n, hw, c) for c, s in cfg])
        torch.cuda.synchronize()
        for j, o in enumerate(outs):
            got[j].append({k: float(v) for k, v in o.items()})
    gotp = [torch.cat([m.optimizer_G.flat_p, m.optimizer_D_A.flat_p, m.optimizer_D_B.flat_p]) for m in run.systems]
    ok = got == want and all(torch.equal(a, b) for a, b in zip(gotp, wantp))
    if not ok:
        first = next(((j, i) for j in range(2) for i in range(steps) if got[j][i] != want[j][i]), None)
        bad.append({"run": r, "first_loss_mismatch": first,
                    "params_equal": [bool(torch.equal(a, b)) for a, b in zip(gotp, wantp)]})
    print(f"run {r}: {'ok' if ok else 'DIVERGED'}", flush=True)
print(json.dumps({"mode": mode, "runs": R, "diverged": len(bad), "detail": bad}))
