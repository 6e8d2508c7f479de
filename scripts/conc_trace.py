"""Locate the first tensor that differs between a sequential and a concurrent (two-stream) run:
clones (on the current stream, so the overlap is kept) of every fused network's inputs,
outputs, incoming gradients and returned gradients, and of each optimizer's flat gradient.
    python scripts/conc_trace.py MODE"""
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_train import _system
from test_gpu_concurrent import _batch
from modules.hip import ops, networks as net
from modules import optim

ops.set_mma(sys.argv[1])
LOG = {"cur": None}


def rec(tag, ts):
    if LOG["cur"] is None:
        return
    for i, t in enumerate(ts):
        if isinstance(t, torch.Tensor) and t.is_cuda:
            LOG["cur"].append((f"{tag}[{i}]", t.detach().clone()))


def wrap(cls, name):
    f0, b0 = cls.forward, cls.backward

    def fwd(ctx, *a):
        rec(f"{name}.fwd.in", a)
        out = f0(ctx, *a)
        rec(f"{name}.fwd.out", [out])
        return out

    def bwd(ctx, *g):
        rec(f"{name}.bwd.dout", g)
        r = b0(ctx, *g)
        rec(f"{name}.bwd.grads", r)
        return r
    cls.forward, cls.backward = staticmethod(fwd), staticmethod(bwd)


wrap(net.GeneratorFunction, "G")
wrap(net.DiscriminatorFunction, "D")
wrap(net.ResBlockFunction, "R")
st0 = optim.FusedAdam.step


def ostep(self, *a, **k):
    rec("adam.flat_g", [self.flat_g])
    return st0(self, *a, **k)


optim.FusedAdam.step = ostep

n, hw, nb, steps = 2, 64, 2, 2
cfg = [(3, 801), (2, 802)]
want = [[], []]
for j, (c, s) in enumerate(cfg):
    m = _system(c, nb, prng.step_model_seeds(s))
    for i in range(steps):
        LOG["cur"] = []
        m.train_step(*_batch(s, i, n, hw, c))
        want[j].append(LOG["cur"])
    torch.cuda.synchronize()
LOG["cur"] = None
sysc = [_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg]
sts = [torch.cuda.Stream(), torch.cuda.Stream()]
got = [[], []]
for i in range(steps):
    cur = torch.cuda.current_stream()
    for j, (m, st, (c, s)) in enumerate(zip(sysc, sts, cfg)):
        b = _batch(s, i, n, hw, c)
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            for t in b:
                t.record_stream(st)
            LOG["cur"] = []
            m.train_step(*b)
            got[j].append(LOG["cur"])
    LOG["cur"] = None
    for st in sts:
        cur.wait_stream(st)
torch.cuda.synchronize()
for j in range(2):
    for i in range(steps):
        W, G = want[j][i], got[j][i]
        assert [k for k, _ in W] == [k for k, _ in G]
        bad = [(idx, k, float((a - b).abs().max())) for idx, ((k, a), (_, b)) in enumerate(zip(W, G))
               if not torch.equal(a, b)]
        print(f"model {j} step {i}: {len(W)} records, {len(bad)} differ; first: {bad[:4]}")
