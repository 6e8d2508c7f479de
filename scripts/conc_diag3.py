"""Localise a concurrent-vs-sequential difference: the flat gradients each optimizer sees at
every step (G, D_A, D_B), per parameter, sequential vs the concurrent schedule.
   python scripts/conc_diag3.py MODE [STEPS]"""
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_train import _system
from test_gpu_concurrent import _batch
from modules.hip import ops
from modules.trainer import ConcurrentCycleGANs

n, hw, nb = 2, 64, 2
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
cfg = [(3, 801), (2, 802)]
ops.set_mma(sys.argv[1])


def instrument(sysm, log):
    for name in ("optimizer_G", "optimizer_D_A", "optimizer_D_B"):
        opt = getattr(sysm, name)
        orig = opt.step

        def step(closure=None, _o=opt, _orig=orig, _n=name):
            log.append((_n, _o.flat_g.clone()))
            return _orig(closure)
        opt.step = step


def names(sysm):
    out = {}
    for oname, mods in (("optimizer_G", (sysm.G_A2B, sysm.G_B2A)), ("optimizer_D_A", (sysm.D_A,)),
                        ("optimizer_D_B", (sysm.D_B,))):
        lst, off = [], 0
        for mi, m in enumerate(mods):
            for pn, p in m.named_parameters():
                lst.append((f"m{mi}.{pn}", off, p.numel()))
                off += p.numel()
        out[oname] = lst
    return out


def attempt():
    seq = [_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg]
    logs_s = [[], []]
    for j, m in enumerate(seq):
        instrument(m, logs_s[j])
    for j, (m, (c, s)) in enumerate(zip(seq, cfg)):
        for i in range(steps):
            m.train_step(*_batch(s, i, n, hw, c))
    torch.cuda.synchronize()
    systems = [_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg]
    logs_c = [[], []]
    for j, m in enumerate(systems):
        instrument(m, logs_c[j])
    run = ConcurrentCycleGANs(systems, "cuda", schedule="concurrent")
    for i in range(steps):
        run.train_step([_batch(s, i, n, hw, c) for c, s in cfg])
    torch.cuda.synchronize()
    found = False
    for j in range(2):
        nm = names(seq[j])
        for k, ((on, gs), (_, gc)) in enumerate(zip(logs_s[j], logs_c[j])):
            if torch.equal(gs, gc):
                continue
            found = True
            bad = []
            for pn, off, cnt in nm[on]:
                a, b = gs[off:off + cnt], gc[off:off + cnt]
                if not torch.equal(a, b):
                    d = (a - b).abs()
                    bad.append(f"{pn}[{int((d > 0).sum())}/{cnt} max {float(d.max()):.3g} "
                               f"rel {float(d.max() / a.abs().max().clamp_min(1e-30)):.3g}]")
            print(f"model {j} call {k} {on}: DIFF", "; ".join(bad[:14]), flush=True)
            break  # the first differing call of this model
    return found


for a in range(int(sys.argv[3]) if len(sys.argv) > 3 else 8):
    if attempt():
        print("difference at attempt", a)
        break
    print("attempt", a, "identical", flush=True)
