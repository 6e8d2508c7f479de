import sys, torch
sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_train import _system
from test_gpu_concurrent import _batch
from modules.hip import ops
for mode in sys.argv[1:]:
    ops.set_mma(mode)
    runs = []
    for r in range(2):
        m = _system(3, 2, prng.step_model_seeds(801))
        runs.append([{k: float(v) for k, v in m.train_step(*_batch(801, i, 2, 64, 3)).items()} for i in range(3)])
    print(mode, "seq-vs-seq identical:", runs[0] == runs[1])
    if runs[0] != runs[1]:
        for a, b in zip(runs[0], runs[1]):
            print({k: (a[k], b[k]) for k in a if a[k] != b[k]})
