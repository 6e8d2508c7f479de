"""Which ingredient of the concurrent schedule changes the numbers?  Against the sequential run
(default stream): (a) two streams overlapping, (b) two streams, each model's step finished
(device sync) before the next model's, (c) one side stream for both models.  Counts, over
ATTEMPTS fresh repetitions, how often the losses of 3 steps differ.
   python scripts/conc_diag4.py MODE ATTEMPTS"""
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
attempts = int(sys.argv[2])


def losses(o):
    return {k: float(v) for k, v in o.items()}


def seq_run():
    seq = [_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg]
    return [[losses(m.train_step(*_batch(s, i, n, hw, c))) for i in range(steps)] for m, (c, s) in zip(seq, cfg)]


def variant(kind):
    systems = [_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg]
    streams = [torch.cuda.Stream() for _ in cfg] if kind != "c" else [torch.cuda.Stream()] * 2
    cur = torch.cuda.current_stream()
    got = [[], []]
    for i in range(steps):
        outs = []
        for sysm, st, (c, s) in zip(systems, streams, cfg):
            b = _batch(s, i, n, hw, c)
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                for t in b:
                    t.record_stream(st)
                outs.append(sysm.train_step(*b))
            if kind in ("b", "c"):
                torch.cuda.synchronize()
        for st in streams:
            cur.wait_stream(st)
        torch.cuda.synchronize()
        for j, o in enumerate(outs):
            got[j].append(losses(o))
    return got


want = seq_run()
for kind in (sys.argv[3].split(",") if len(sys.argv) > 3 else ("a", "b", "c")):
    bad = 0
    for a in range(attempts):
        g = variant(kind)
        if g != want:
            bad += 1
            which = [(j, i) for j in range(2) for i in range(steps) if g[j][i] != want[j][i]]
            print(f"  variant {kind} attempt {a}: differs at (model, step) {which}", flush=True)
    print(f"variant {kind}: {bad}/{attempts} attempts differ", flush=True)
