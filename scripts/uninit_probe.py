"""Reads of never-written device memory: fill the caching allocator's free blocks with a
pattern (0, then NaN, then 3.7e19) before every train step of fresh systems on one stream and
compare the losses of 3 steps.  Any dependence on the pattern is a read of memory no kernel
wrote.   python scripts/uninit_probe.py MODE"""
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_train import _system
from test_gpu_concurrent import _batch
from modules.hip import ops

n, hw, nb, steps = 2, 64, 2, 3
cfg = [(3, 801), (2, 802)]
ops.set_mma(sys.argv[1])


def fill_pool(val):
    blocks = []
    for k in range(8, 27):  # 256 B .. 64 MiB, a few of each
        for _ in range(6):
            blocks.append(torch.full((2 ** k // 4,), val, device="cuda"))
    torch.cuda.synchronize()
    del blocks


def run(val):
    out = []
    for c, s in cfg:
        m = _system(c, nb, prng.step_model_seeds(s))
        seq = []
        for i in range(steps):
            b = _batch(s, i, n, hw, c)
            fill_pool(val)
            seq.append({k: float(v) for k, v in m.train_step(*b).items()})
        out.append(seq)
    return out


base = run(0.0)
for val in (float("nan"), 3.7e19, -1.0):
    got = run(val)
    same = got == base
    print(f"pattern {val}: identical {same}", flush=True)
    if not same:
        for j in range(2):
            for i in range(steps):
                d = {k: (base[j][i][k], got[j][i][k]) for k in base[j][i] if base[j][i][k] != got[j][i][k]}
                if d:
                    print(f"  model {j} step {i}:", {k: f"{a:.7g} vs {b:.7g}" for k, (a, b) in list(d.items())[:4]})
