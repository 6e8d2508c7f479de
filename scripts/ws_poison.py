"""Does any op read workspace bytes it did not write?  Runs 3 train steps per model and mode,
prints the losses; run once with DUCOSY_WS_POISON=1 (scratch filled with NaN bytes on every
request) and once without, and compare."""
import json
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_train import _system
from test_gpu_concurrent import _batch
from modules.hip import ops

res = {}
for mode in sys.argv[1:]:
    ops.set_mma(mode)
    for c, s in [(3, 801), (2, 802)]:
        m = _system(c, 2, prng.step_model_seeds(s))
        res[f"{mode}/{c}"] = [{k: float(v) for k, v in m.train_step(*_batch(s, i, 2, 64, c)).items()} for i in range(3)]
print(json.dumps(res))
