"""Concurrent vs sequential: after each step, which parameters of which model differ first.
    python scripts/conc_params.py MODE [serial]"""
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_train import _system
from test_gpu_concurrent import _batch
from modules.hip import ops

mode = sys.argv[1]
serial = len(sys.argv) > 2 and sys.argv[2] == "serial"
ops.set_mma(mode)
n, hw, nb, steps = 2, 64, 2, 3
cfg = [(3, 801), (2, 802)]


def snap(s):
    out = {}
    for name, m in zip(("G_A2B", "G_B2A", "D_A", "D_B"), s.models):
        for k, p in m.named_parameters():
            out[f"{name}.{k}"] = p.detach().clone()
    return out


seq = [_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg]
want = [[], []]
for j, (m, (c, s)) in enumerate(zip(seq, cfg)):
    for i in range(steps):
        m.train_step(*_batch(s, i, n, hw, c))
        torch.cuda.synchronize()
        want[j].append(snap(m))
sysc = [_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg]
sts = [torch.cuda.Stream(), torch.cuda.Stream()]
got = [[], []]
for i in range(steps):
    cur = torch.cuda.current_stream()
    prev = None
    for j, (m, st, (c, s)) in enumerate(zip(sysc, sts, cfg)):
        b = _batch(s, i, n, hw, c)
        st.wait_stream(cur)
        if serial and prev is not None:
            st.wait_stream(prev)
        with torch.cuda.stream(st):
            for t in b:
                t.record_stream(st)
            m.train_step(*b)
        prev = st
    for st in sts:
        cur.wait_stream(st)
    torch.cuda.synchronize()
    for j in range(2):
        got[j].append(snap(sysc[j]))
print(mode, "serial" if serial else "overlap")
for j in range(2):
    for i in range(steps):
        bad = [(k, float((want[j][i][k] - got[j][i][k]).abs().max())) for k in want[j][i]
               if not torch.equal(want[j][i][k], got[j][i][k])]
        if bad:
            print(f"  model {j} step {i}: {len(bad)} params differ; first: {bad[:6]}")
            break
    else:
        print(f"  model {j}: identical")
