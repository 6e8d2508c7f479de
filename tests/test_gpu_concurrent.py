"""BASELINE config 5 on one GPU: the soft-tissue (cin 3) and lung (cin 2) CycleGANs trained in one
process (modules/trainer.py ConcurrentCycleGANs, serial schedule; the reference trains them one
after the other, train.py:27-38).

* each model gets exactly the losses and weights of its own run, in the default operand mode and
  in config 5's fp16 MFMA mode (the kernels are deterministic; the models share only workspaces);
* in the fp16 mode both models of the pair hold the fp16 bar of tests/test_gpu_train.py (5e-3 on
  step-0 losses, the 1e-2 envelope after): the soft-tissue model against the reference-generated
  step fixture (tests/golden/steps_64.npz), the lung model against the oracle (no reference
  fixture has a cin-2 step).  One exception: the lung model's ContrastEdge term after two Adam
  steps is held to 2e-2 of its scale (measured 1.2e-2).  Its top-10 % edge set and the |std p -
  std t| cancellation make it the term most sensitive to rounding (by step 19 the reference's own
  runs at different thread counts spread 40 % on it, tests/test_gpu_curve.py), and each of Adam's
  first updates is lr * sign(g), which fp16 operands flip for gradients near zero."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import prng
from oracle import ref_torch as orc
from test_gpu_train import _sd, _system

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _batch(seed, i, n, hw, cin):
    rA = torch.from_numpy(prng.uniform(seed, f"A{i}", (n, 1, hw, hw), -1, 1)).to(DEV)
    rB = torch.from_numpy(prng.uniform(seed, f"B{i}", (n, 1, hw, hw), -1, 1)).to(DEV)
    mk = torch.from_numpy(prng.bernoulli(seed, f"M{i}", (n, cin - 1, hw, hw), 0.3)).to(DEV)
    return rA, rB, mk


@pytest.mark.parametrize("mode", ["f16x3", "f16"])
def test_serial_schedule_equals_independent_runs(mode):
    """The serial schedule (both models on the caller's stream) gives each model exactly the numbers
    of its own run."""
    from modules.hip import ops
    from modules.trainer import ConcurrentCycleGANs
    n, hw, nb, steps = 2, 64, 2, 2
    cfg = [(3, 811), (2, 812)]
    prev = ops.get_mma()
    ops.set_mma(mode)
    try:
        want = []
        for c, s in cfg:
            m = _system(c, nb, prng.step_model_seeds(s))
            want.append([{k: float(v) for k, v in m.train_step(*_batch(s, i, n, hw, c)).items()}
                         for i in range(steps)])
        run = ConcurrentCycleGANs([_system(c, nb, prng.step_model_seeds(s)) for c, s in cfg], DEV)
        got = [[], []]
        for i in range(steps):
            for j, o in enumerate(run.train_step([_batch(s, i, n, hw, c) for c, s in cfg])):
                got[j].append({k: float(v) for k, v in o.items()})
        assert got == want
    finally:
        ops.set_mma(prev)


def test_dual_f16_vs_reference():
    from modules.hip import ops
    from modules.trainer import ConcurrentCycleGANs
    z = np.load(os.path.join(GOLDEN, "steps_64.npz"))
    n, hw, nb, cin, steps, seed = [int(v) for v in z["meta"]]
    lung_seed = 813
    ls = prng.step_model_seeds(lung_seed)
    gs, ds = orc.generator_param_shapes(2, nb, True), orc.discriminator_param_shapes(1)
    oracle = orc.OracleCycleGAN(_sd(gs, ls["G_A2B"]), _sd(gs, ls["G_B2A"]), _sd(ds, ls["D_A"]),
                                _sd(ds, ls["D_B"]), nb)
    prev = ops.get_mma()
    ops.set_mma("f16")
    try:
        run = ConcurrentCycleGANs([_system(cin, nb, prng.step_model_seeds(seed)),
                                   _system(2, nb, ls)], DEV)
        lung0 = None
        for i in range(steps):
            soft = _batch(seed, i, n, hw, cin)
            lung = _batch(lung_seed, i, n, hw, 2)
            want_lung = oracle.step(*(t.cpu() for t in lung))
            lung0 = lung0 or want_lung
            out_soft, out_lung = ({k: float(v) for k, v in o.items()} for o in run.train_step([soft, lung]))
            tol = 5e-3 if i == 0 else 1e-2
            for k, v in out_soft.items():
                ref = float(z[k][i])
                scale = ref if i == 0 else max(abs(ref), abs(float(z[k][0])))
                assert abs(v - ref) <= tol * max(abs(scale), 1e-2), ("soft", i, k, v, ref)
            for k, v in out_lung.items():
                ref = want_lung[k]
                scale = max(abs(ref), abs(lung0[k]))  # a term may shrink to a near-cancellation
                tk = 2e-2 if (k == "loss_contrast_edge" and i >= 2) else tol
                assert abs(v - ref) <= tk * max(scale, 1e-2), ("lung", i, k, v, ref)
    finally:
        ops.set_mma(prev)
