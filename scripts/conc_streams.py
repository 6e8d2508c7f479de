"""Which HIP stream does every kernel of a concurrent two-model step run on?  Run under
rocprofv3 --kernel-trace: two systems step once on two side streams (bf16x6), after a marker
fill on each stream so the trace can name them.
   rocprofv3 --kernel-trace --output-format csv -d DIR -- python scripts/conc_streams.py MODE"""
import sys

import torch

sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_train import _system
from test_gpu_concurrent import _batch
from modules.hip import ops

ops.set_mma(sys.argv[1] if len(sys.argv) > 1 else "bf16x6")
n, hw, nb = 2, 64, 2
cfg = [(3, 801), (2, 802)]
batches = [_batch(s, 0, n, hw, c) for c, s in cfg]
systems = [_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg]
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
marks = [torch.empty(1 << 16, device="cuda") for _ in cfg]
torch.cuda.synchronize()
cur = torch.cuda.current_stream()
for rep in range(2):
    for j, (sysm, st) in enumerate(zip(systems, streams)):
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            marks[j].fill_(float(j + 1))  # FillFunctor on stream j: names the stream in the trace
            for t in batches[j]:
                t.record_stream(st)
            sysm.train_step(*batches[j])
    for st in streams:
        cur.wait_stream(st)
    torch.cuda.synchronize()
print("streams", [s.cuda_stream for s in streams], "null", cur.cuda_stream, flush=True)
