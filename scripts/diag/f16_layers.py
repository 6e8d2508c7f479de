"""Which window phase-kernel layers (and, with --fixed, which stem / head kernels) can run on fp16 operands in config 5's fp16 mode: the f16 soft +
lung pair (tests/test_gpu_concurrent.py::test_dual_f16_vs_reference) with ops._PHASE_F16X3 narrowed,
printing per variant the largest deviation of every loss term as a fraction of that test's bar (<= 1
passes).   python scripts/diag/f16_layers.py"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "ducosy-gan_amd")]
import numpy as np  # noqa: E402

from conftest import GOLDEN  # noqa: E402
from oracle import prng  # noqa: E402
from oracle import ref_torch as orc  # noqa: E402
from test_gpu_concurrent import _batch  # noqa: E402
from test_gpu_train import _sd, _system  # noqa: E402
from modules.hip import ops  # noqa: E402
from modules.trainer import ConcurrentCycleGANs  # noqa: E402

ALL = ("up1", "up2", "pg64", "pg128", "pg256")


def run(keep, fixed=("stem", "stem_wgrad", "head")):
    ops._PHASE_F16X3 = frozenset(keep)
    ops._FIXED_F16X3 = frozenset(fixed)
    z = np.load(os.path.join(GOLDEN, "steps_64.npz"))
    n, hw, nb, cin, steps, seed = [int(v) for v in z["meta"]]
    lung_seed = 813
    ls = prng.step_model_seeds(lung_seed)
    gs, ds = orc.generator_param_shapes(2, nb, True), orc.discriminator_param_shapes(1)
    oracle = orc.OracleCycleGAN(_sd(gs, ls["G_A2B"]), _sd(gs, ls["G_B2A"]), _sd(ds, ls["D_A"]),
                                _sd(ds, ls["D_B"]), nb)
    ops.set_mma("f16")
    run_ = ConcurrentCycleGANs([_system(cin, nb, prng.step_model_seeds(seed)), _system(2, nb, ls)], "cuda")
    worst = {}
    lung0 = None
    for i in range(steps):
        soft = _batch(seed, i, n, hw, cin)
        lung = _batch(lung_seed, i, n, hw, 2)
        want_lung = oracle.step(*(t.cpu() for t in lung))
        lung0 = lung0 or want_lung
        out_soft, out_lung = ({k: float(v) for k, v in o.items()} for o in run_.train_step([soft, lung]))
        tol = 5e-3 if i == 0 else 1e-2
        for k, v in out_soft.items():
            ref = float(z[k][i])
            scale = ref if i == 0 else max(abs(ref), abs(float(z[k][0])))
            r = abs(v - ref) / (tol * max(abs(scale), 1e-2))
            worst[("soft", k)] = max(worst.get(("soft", k), 0.0), r)
        for k, v in out_lung.items():
            ref = want_lung[k]
            scale = max(abs(ref), abs(lung0[k]))
            tk = 2e-2 if (k == "loss_contrast_edge" and i >= 2) else tol
            r = abs(v - ref) / (tk * max(scale, 1e-2))
            worst[("lung", k)] = max(worst.get(("lung", k), 0.0), r)
    return worst


if __name__ == "__main__":
    if "--fixed" in sys.argv:  # the stem / head kernels (ops._FIXED_F16X3), phase layers all on fp16
        FX = ("stem", "stem_wgrad", "head")
        for fixed in (FX, (), ("stem", "head"), ("stem",), ("head",), ("stem", "stem_wgrad")):
            w = run((), fixed)
            top = sorted(w.items(), key=lambda kv: -kv[1])[:3]
            print(f"f16x3 kernels {list(fixed)}: max {max(w.values()):.2f}  " +
                  "  ".join(f"{m}/{k.replace('loss_', '')} {r:.2f}" for (m, k), r in top), flush=True)
        sys.exit(0)
    variants = [ALL, ()] + [tuple(x for x in ALL if x != d) for d in ALL]
    for keep in variants:
        w = run(keep)
        top = sorted(w.items(), key=lambda kv: -kv[1])[:3]
        f16 = sorted(set(ALL) - set(keep))
        print(f"f16 layers {f16}: max {max(w.values()):.2f}  " +
              "  ".join(f"{m}/{k.replace('loss_', '')} {r:.2f}" for (m, k), r in top), flush=True)
