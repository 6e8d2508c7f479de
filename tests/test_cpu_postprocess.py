"""modules/postprocess.py (drop-in for the reference's modules/postprocess.py) against outputs the
reference module itself produced (tests/golden/make_golden_post.py), and generate.py's
synthesis smoothing (modules/inference.py::smooth_volume) against the reference's own
two-stage call (generate.py:246-254)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def z():
    return np.load(os.path.join(GOLDEN, "postprocess.npz"))


CASES = {
    "gaussian": dict(method="gaussian"),
    "gaussian_s2": dict(method="gaussian", sigma=2.0, enhance_sharpness=False),
    "gaussian3d": dict(method="gaussian3d"),
    "gaussian3d_synth": dict(method="gaussian3d", sigma_z=0.7, sigma_xy=0.05, enhance_sharpness=True,
                             sharpen_amount=1.7, sharpen_radius=1.2),
    "adaptive": dict(method="adaptive"),
    "median": dict(method="median", enhance_sharpness=False),
    "median5": dict(method="median", kernel_size=5),
    "interpolation": dict(method="interpolation"),
    "kalman": dict(method="kalman"),
    "kalman_q": dict(method="kalman", process_variance=1e-3, measurement_variance=1e-1, enhance_sharpness=False),
    "thr500": dict(method="gaussian3d", hu_threshold=500),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_postprocess_ct_volume_matches_reference(z, name):
    from modules.postprocess import postprocess_ct_volume
    got = postprocess_ct_volume(z["volume"].copy(), **CASES[name])
    want = z[f"post:{name}"]
    assert got.dtype == want.dtype == np.int16
    assert np.array_equal(got, want), (name, int(np.abs(got.astype(int) - want).max()))


def test_helpers_match_reference(z):
    from modules import postprocess as pp
    assert np.array_equal(pp.unsharp_mask(z["volume2"], z["volume"], amount=0.8, radius=1.5), z["unsharp"])
    assert np.array_equal(pp.kalman_filter_1d(z["volume"][:, 3, 3].astype(np.float64), 1e-5, 1e-2), z["kalman1d"])
    d = z["diff"].copy()
    assert np.array_equal(pp.apply_diffmap(z["volume"].copy(), d, threshold=8), z["diffmap"])
    assert d.min() == 0 or d.min() >= 8  # thresholded in place, as the reference


def test_unknown_method_raises(z):
    from modules.postprocess import postprocess_ct_volume
    with pytest.raises(ValueError):
        postprocess_ct_volume(z["volume"], method="bilateral")


def test_synthesis_smoothing_matches_reference(z):
    from modules.inference import smooth_volume
    assert np.array_equal(smooth_volume(z["volume"]), z["synth"])
