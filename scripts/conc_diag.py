"""Concurrent-vs-sequential diagnostics (tests/test_gpu_concurrent.py setting): per model and
step, the losses that differ and by how much.   python scripts/conc_diag.py MODE [MODE ...]"""
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_train import _system
from test_gpu_concurrent import _batch
from modules.hip import ops
from modules.trainer import ConcurrentCycleGANs

n, hw, nb, steps = 2, 64, 2, 3
cfg = [(3, 801), (2, 802)]
for mode in sys.argv[1:]:
    ops.set_mma(mode)
    seq = [_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg]
    want = [[{k: float(v) for k, v in m.train_step(*_batch(s, i, n, hw, c)).items()} for i in range(steps)]
            for m, (c, s) in zip(seq, cfg)]
    run = ConcurrentCycleGANs([_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg], "cuda")
    got = [[], []]
    for i in range(steps):
        outs = run.train_step([_batch(s, i, n, hw, c) for c, s in cfg])
        torch.cuda.synchronize()
        for j, o in enumerate(outs):
            got[j].append({k: float(v) for k, v in o.items()})
    print(mode, "identical:", got == want)
    for j in range(2):
        for i in range(steps):
            d = {k: (want[j][i][k], got[j][i][k]) for k in want[j][i] if want[j][i][k] != got[j][i][k]}
            if d:
                print(f"  model {j} step {i}:", {k: f"{a:.7g} vs {b:.7g}" for k, (a, b) in d.items()})
