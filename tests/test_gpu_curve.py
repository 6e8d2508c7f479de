"""Loss-curve parity: 50 training steps of CycleGANSystem (HIP, default f16x3 operands) at
BASELINE config 1 (128x128, bs 2, 1 residual block, cin 3) against the reference's own step loop
(modules/trainer.py:447-525, tests/golden/make_golden.py --curve) run at 1, 2, 3, 4, 6 and 8 torch
threads.

The reference does not agree with itself across thread counts: summation order changes the
rounding, Adam turns rounding into +-lr moves, and the GAN game amplifies them (by step 19 the
runs spread by 40 % on the contrast-edge term).  The bar is therefore calibrated on the reference
runs themselves.  For a curve g and a set of reference runs r, at every step and for every one of
the 12 loss terms,

    q = |g - median(r)| / (spread(r) + FLOOR * |median(r)|)

with spread the largest max-min of the runs up to that step and FLOOR = 1e-3 (north_star's
forward tolerance).  Q_ref = the largest q of any reference run judged against the other five
(leave-one-out); the HIP curve, judged against all six, must stay within it at every step.  So the
HIP run deviates no more than the reference's own most deviant run does.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import prng

from conftest import GOLDEN, ROOT
from test_gpu_train import _system

pytestmark = pytest.mark.gpu
DEV = "cuda"
FLOOR = 1e-3


def _q(g, r):
    """Deviation of curve g from runs r ([runs, steps]) in units of their running spread."""
    mid = np.median(r, 0)
    env = np.maximum.accumulate(r.max(0) - r.min(0))
    return np.abs(g - mid) / (env + FLOOR * np.abs(mid))


def test_loss_curve_within_reference_spread():
    z = np.load(os.path.join(GOLDEN, "curve_128.npz"))
    n, hw, nb, cin, steps, seed = [int(v) for v in z["meta"]]
    threads = [int(t) for t in z["threads"]]
    keys = [k.split(":", 1)[1] for k in z.files if k.startswith(f"t{threads[0]}:")]
    ref = {k: np.stack([z[f"t{t}:{k}"] for t in threads]) for k in keys}  # [runs, steps]
    s = _system(cin, nb, prng.step_model_seeds(seed))
    got = {k: [] for k in keys}
    for i in range(steps):
        rA = torch.from_numpy(prng.uniform(seed, f"A{i}", (n, 1, hw, hw), -1, 1)).to(DEV)
        rB = torch.from_numpy(prng.uniform(seed, f"B{i}", (n, 1, hw, hw), -1, 1)).to(DEV)
        mk = torch.from_numpy(prng.bernoulli(seed, f"M{i}", (n, cin - 1, hw, hw), 0.3)).to(DEV)
        out = s.train_step(rA, rB, mk)
        for k in keys:
            got[k].append(float(out[k]))
    q_ref = 0.0  # leave-one-out: each reference run against the others
    for i in range(len(threads)):
        for k in keys:
            q_ref = max(q_ref, float(_q(ref[k][i], np.delete(ref[k], i, 0)).max()))
    report, bad = {"q_ref": q_ref}, []
    for k in keys:
        r = ref[k]
        g = np.array(got[k])
        q = _q(g, r)
        report[k] = {"hip": g.tolist(), "ref_median": np.median(r, 0).tolist(),
                     "ref_spread": (r.max(0) - r.min(0)).tolist(), "q_max": float(q.max()),
                     "q_mean": float(q.mean())}
        for i in np.nonzero(q > q_ref)[0][:3]:
            bad.append((k, int(i), float(g[i]), float(np.median(r[:, i])), float(q[i]), q_ref))
    out_dir = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out_dir):
        with open(os.path.join(out_dir, "curve_hip.json"), "w") as f:
            json.dump(report, f)
    assert q_ref >= 1.0, q_ref  # the reference runs do spread
    assert not bad, bad
