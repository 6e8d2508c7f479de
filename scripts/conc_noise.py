"""Is the concurrent-schedule difference an interaction between the two models, or does any
co-running work perturb one model's kernels?  Model (cin 2) trains on a side stream while a
second side stream runs unrelated noise work; its losses are compared with a sequential run.
   python scripts/conc_noise.py MODE ATTEMPTS NOISE   (NOISE: matmul | rows | none)"""
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_train import _system
from test_gpu_concurrent import _batch
from modules.hip import ops
from modules.hip.lib import DCS_PAD_REFLECT

n, hw, nb, steps = 2, 64, 2, 3
c, s = 2, 802
ops.set_mma(sys.argv[1])
attempts, noise = int(sys.argv[2]), sys.argv[3]


def losses(o):
    return {k: float(v) for k, v in o.items()}


m = _system(c, nb, prng.step_model_seeds(s))
want = [losses(m.train_step(*_batch(s, i, n, hw, c))) for i in range(steps)]
A = torch.randn(2048, 2048, device="cuda")
g = ops.ConvGeom(256, 256, 3, 1, (1, 1, 1, 1), DCS_PAD_REFLECT)
x = torch.randn(8, 64, 64, 256, device="cuda")
wp = g.pack_fwd(torch.randn(256, 256, 3, 3, device="cuda") * 0.02)
torch.cuda.synchronize()
bad = 0
for a in range(attempts):
    m = _system(c, nb, prng.step_model_seeds(s))
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    cur = torch.cuda.current_stream()
    got = []
    for i in range(steps):
        b = _batch(s, i, n, hw, c)
        sa.wait_stream(cur)
        sb.wait_stream(cur)
        with torch.cuda.stream(sb):
            for _ in range(int(sys.argv[4]) if len(sys.argv) > 4 else 40):
                if noise == "matmul":
                    A = torch.tanh(A @ A * 1e-3)
                elif noise == "rows":
                    g.forward(ops.Src.nhwc(x), wp)
                elif noise == "dgrad":
                    g.dgrad(x, wp, 64, 64)
                elif noise == "wgrad":
                    g.wgrad(x, ops.Src.nhwc(x))
        with torch.cuda.stream(sa):
            for t in b:
                t.record_stream(sa)
            out = m.train_step(*b)
        cur.wait_stream(sa)
        cur.wait_stream(sb)
        torch.cuda.synchronize()
        got.append(losses(out))
    if got != want:
        bad += 1
        print(f"  attempt {a}: steps differing {[i for i in range(steps) if got[i] != want[i]]}", flush=True)
print(f"noise {noise}: {bad}/{attempts} attempts differ", flush=True)
