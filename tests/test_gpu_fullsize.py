"""Parity at the north-star size (BASELINE config 3: 512 x 512, 9 residual blocks, cin 3):
  * two full training steps of one slice on the GPU against the CPU oracle (oracle/ref_torch.py,
    pinned to the reference by the golden fixtures at small sizes): every loss term within the
    golden test's bars (1e-3 at step 0, whose losses are pure forward; 1e-2 after one Adam
    update, which carries the gradients);
  * at bs 8: the default bf16x6 mode is bit-reproducible and within 1e-4 of the exact-f32
    path on every loss term (both are fp32-class; the difference is accumulation order)."""
import pytest
import torch

from oracle import prng
from oracle import ref_torch as orc
from test_gpu_train import _system

pytestmark = pytest.mark.gpu
DEV = "cuda"
HW, NB, CIN = 512, 9, 3


def _inputs(seed, i, n):
    a = torch.from_numpy(prng.uniform(seed, f"A{i}", (n, 1, HW, HW), -1, 1))
    b = torch.from_numpy(prng.uniform(seed, f"B{i}", (n, 1, HW, HW), -1, 1))
    m = torch.from_numpy(prng.bernoulli(seed, f"M{i}", (n, CIN - 1, HW, HW), 0.3))
    return a, b, m


def _rel(v, ref):
    return abs(v - ref) / max(abs(ref), 1e-2)


def test_fullsize_steps_match_oracle():
    from modules.hip import ops
    seed = 901
    seeds = prng.step_model_seeds(seed)
    torch.set_num_threads(16)
    sd = lambda shapes, s: {k: torch.from_numpy(v) for k, v in prng.init_state_dict(shapes, s).items()}
    gs, ds = orc.generator_param_shapes(CIN, NB, True), orc.discriminator_param_shapes(1)
    oracle = orc.OracleCycleGAN(sd(gs, seeds["G_A2B"]), sd(gs, seeds["G_B2A"]), sd(ds, seeds["D_A"]),
                                sd(ds, seeds["D_B"]), NB)
    gpu = _system(CIN, NB, seeds)
    worst = {}
    for i in range(2):
        a, b, m = _inputs(seed, i, 1)
        want = oracle.step(a, b, m)
        got = {k: float(v) for k, v in gpu.train_step(a.to(DEV), b.to(DEV), m.to(DEV)).items()}
        # step 1 follows one Adam update (measured 2.9e-4; the CPU reference itself moves ~2e-4 on the
        # D losses across thread counts after one step)
        tol = 1e-3 if i == 0 else 2e-3
        for k, ref in want.items():
            e = _rel(got[k], float(ref))
            worst[(i, k)] = e
            assert e <= tol, (ops.get_mma(), i, k, got[k], float(ref), e)
    print("fullsize vs oracle, worst relative error per step:",
          {i: max(v for (j, _), v in worst.items() if j == i) for i in range(2)})


def test_fullsize_bf16x6_deterministic_and_close_to_f32():
    from modules.hip import ops
    seed = 902
    seeds = prng.step_model_seeds(seed)
    a, b, m = (x.to(DEV) for x in _inputs(seed, 0, 8))
    prev = ops.get_mma()
    out = {}
    try:
        for tag, mode in (("x6", "bf16x6"), ("x6b", "bf16x6"), ("f32", "f32")):
            ops.set_mma(mode)
            s = _system(CIN, NB, seeds)
            out[tag] = {k: float(v) for k, v in s.train_step(a, b, m).items()}
            del s
            torch.cuda.empty_cache()
    finally:
        ops.set_mma(prev)
    assert out["x6"] == out["x6b"]
    for k, v in out["f32"].items():
        assert _rel(out["x6"][k], v) <= 1e-4, (k, out["x6"][k], v)
