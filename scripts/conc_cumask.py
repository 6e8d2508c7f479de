"""Does the two-stream difference need the two models' workgroups on the SAME compute units?
Against the sequential run (default stream), counts over ATTEMPTS fresh repetitions how often
the losses of 3 steps differ when the two models run on
  t: two torch side streams (the concurrent schedule as shipped before),
  u: two CU-mask streams that both cover every CU (same stream type as m, no partition),
  m: two CU-mask streams over disjoint halves of the CUs (dcs_stream_create_cu_mask),
  g / e: disjoint CU sets interleaved in blocks of 8 / alternating CUs,
  q: two CU-mask streams sharing a quarter of the CUs.
Batches are made before the loop, and the whole script runs on a torch side stream, so the
legacy null stream (with which CU-mask streams, created blocking, would synchronise) carries no
work.  Events on each model's stream report whether the two steps overlapped in time.
   python scripts/conc_cumask.py MODE ATTEMPTS [VARIANTS]"""
import ctypes
import sys

import torch

sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_train import _system
from test_gpu_concurrent import _batch
from modules.hip import ops, lib

n, hw, nb, steps = 2, 64, 2, 3
cfg = [(3, 801), (2, 802)]
ops.set_mma(sys.argv[1])
attempts = int(sys.argv[2])
L = lib.load()
ncu = L.dcs_device_cu_count()
words = (ncu + 31) // 32


def mask_stream(lo, hi, pick=None):
    m = (ctypes.c_uint32 * words)()
    for i in range(lo, hi):
        if pick is None or pick(i):
            m[i // 32] |= 1 << (i % 32)
    s = ctypes.c_void_p()
    lib.call("dcs_stream_create_cu_mask", m, words, ctypes.byref(s))
    return torch.cuda.ExternalStream(s.value)


def losses(o):
    return {k: float(v) for k, v in o.items()}


MAIN = torch.cuda.Stream()
torch.cuda.set_stream(MAIN)  # nothing on the null stream from here on
batches = [[_batch(s, i, n, hw, c) for i in range(steps)] for c, s in cfg]
seq = [_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg]
want = [[losses(m.train_step(*batches[j][i])) for i in range(steps)] for j, m in enumerate(seq)]
del seq
streams = {"t": [torch.cuda.Stream(), torch.cuda.Stream()],
           "u": [mask_stream(0, ncu), mask_stream(0, ncu)],
           "m": [mask_stream(0, ncu // 2), mask_stream(ncu // 2, ncu)],
           # no CU shared, but each model spread over every block of 8 / every pair of CUs
           "g": [mask_stream(0, ncu, lambda i: (i // 8) % 2 == 0), mask_stream(0, ncu, lambda i: (i // 8) % 2 == 1)],
           "e": [mask_stream(0, ncu, lambda i: i % 2 == 0), mask_stream(0, ncu, lambda i: i % 2 == 1)],
           # the two models share a quarter of the CUs
           "q": [mask_stream(0, 5 * ncu // 8), mask_stream(3 * ncu // 8, ncu)]}
print(f"{ncu} CUs; mode {sys.argv[1]}", flush=True)


OVER = {}


def variant(kind):
    systems = [_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg]
    torch.cuda.synchronize()
    sts = streams[kind]
    cur = torch.cuda.current_stream()
    got = [[], []]
    for i in range(steps):
        outs, ev = [], []
        for j, (sysm, st) in enumerate(zip(systems, sts)):
            b = batches[j][i]
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for t in b:
                    t.record_stream(st)
                outs.append(sysm.train_step(*b))
                e1.record(st)
                ev.append((e0, e1))
        for st in sts:
            cur.wait_stream(st)
        torch.cuda.synchronize()
        (a0, a1), (b0, b1) = ev
        # model 1 starts before model 0 ends (times relative to model 0's start)
        OVER.setdefault(kind, []).append(a0.elapsed_time(b0) < a0.elapsed_time(a1))
        for j, o in enumerate(outs):
            got[j].append(losses(o))
    return got


import time
res, secs = {}, {}
kinds = sys.argv[3].split(",") if len(sys.argv) > 3 else ["t", "u", "m"]
for a in range(attempts):  # interleaved, so drift over the run hits every variant alike
    for kind in kinds:
        t0 = time.perf_counter()
        g = variant(kind)
        secs[kind] = secs.get(kind, 0.0) + time.perf_counter() - t0
        if g != want:
            which = [(j, i) for j in range(2) for i in range(steps) if g[j][i] != want[j][i]]
            print(f"  variant {kind} attempt {a}: differs at (model, step) {which}", flush=True)
            res[kind] = res.get(kind, 0) + 1
for kind in kinds:
    print(f"variant {kind}: {res.get(kind, 0)}/{attempts} attempts differ ({secs[kind] / attempts:.3f} s per attempt; "
          f"steps overlapping {sum(OVER[kind])}/{len(OVER[kind])})",
          flush=True)
