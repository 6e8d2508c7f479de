"""GPU parity of the input-pipeline kernels (dcs_hu_transform, dcs_anatomical_masks) through the
C-ABI: bit-exact masks against the reference's own outputs (tests/golden/masks_*.npz) and the
oracle (oracle/masks_ref.py) on the reference's edge cases (one lung / tiny lungs / empty slice
gating, HU values exactly on every threshold, collinear lungs where qhull raises, ragged sizes,
random component soups), HU transform against the reference's fixture and the oracle."""
import numpy as np
import pytest
import torch

from modules import phantom
from modules.hip import ops
from oracle import masks_ref
from test_cpu_masks import KINDS, _golden, unpack

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _hu_dev(raw, slope, inter):
    hu, _ = ops.hu_transform(torch.from_numpy(raw).to(DEV), torch.from_numpy(slope).to(DEV),
                             torch.from_numpy(inter).to(DEV), -150, 250, want_img=False)
    return hu


@pytest.mark.parametrize("name", ["masks_128", "masks_512"])
def test_masks_match_reference_golden(golden_dir, name):
    z, raw, slope, inter = _golden(golden_dir, name)
    hu = _hu_dev(raw, slope, inter)
    got = ops.anatomical_masks(hu, KINDS, min_size=int(z["min_size"]), border_margin=int(z["border"])).cpu().numpy()
    for i in range(raw.shape[0]):
        for c, k in enumerate(KINDS):
            want = unpack(z, i, c)
            bad = int((got[i, c] != want).sum())
            assert bad == 0, f"slice {i} {k}: {bad} pixels differ"


def test_mask_channel_order_and_subsets(golden_dir):
    """mask_types order = output channel order (dataset.py:135-158): soft-tissue ['bone',
    'mediastinum'] and lung ['lung'] (argmanager.py:132, 149)."""
    z, raw, slope, inter = _golden(golden_dir, "masks_512")
    hu = _hu_dev(raw, slope, inter)
    soft = ops.anatomical_masks(hu, ["bone", "mediastinum"]).cpu().numpy()
    lung = ops.anatomical_masks(hu, ["lung"]).cpu().numpy()
    ves = ops.anatomical_masks(hu, ["lung_vessel"]).cpu().numpy()
    for i in range(raw.shape[0]):
        np.testing.assert_array_equal(soft[i, 0], unpack(z, i, 2))
        np.testing.assert_array_equal(soft[i, 1], unpack(z, i, 1))
        np.testing.assert_array_equal(lung[i, 0], unpack(z, i, 0))
        np.testing.assert_array_equal(ves[i, 0], unpack(z, i, 3))


def _check_vs_oracle(hu_np, **kw):
    got = ops.anatomical_masks(torch.from_numpy(hu_np).to(DEV), KINDS, **kw).cpu().numpy()
    want = masks_ref.masks_batch(hu_np, KINDS, **kw)
    for i in range(hu_np.shape[0]):
        for c, k in enumerate(KINDS):
            bad = int((got[i, c] != want[i, c]).sum())
            assert bad == 0, f"slice {i} {k}: {bad} pixels differ"


def test_masks_ragged_sizes_vs_oracle():
    """Non-square, non-power-of-two slices (W not a multiple of the 64-lane wave)."""
    for (H, W) in ((96, 100), (130, 77)):
        hu = np.stack([phantom.slice_hu(31, i, max(H, W))[:H, :W] for i in range(5)]).astype(np.float32)
        _check_vs_oracle(hu, min_size=16, border_margin=6)


def test_masks_collinear_lungs_fallback():
    """All lung pixels on one row: qhull raises, the reference falls back (hull = lung mask for
    the mediastinum, no exclusion for bone)."""
    hu = np.full((1, 64, 64), -1024.0, np.float32)
    hu[0, 30, 10:28] = -800
    hu[0, 30, 34:54] = -800
    hu[0, 40:44, 20:30] = 300       # bone candidates inside the body
    hu[0, 29, 10:54] = 20           # a thin body so the lung/body ratio passes
    _check_vs_oracle(hu, min_size=8, border_margin=4)


def test_masks_threshold_values_exact():
    """HU exactly at -1000, -300, 200, 450, 600 on and around lungs, hull vertices at -300."""
    hu = np.stack([phantom.slice_hu(41, 4, 192, kind="edges") for _ in range(2)]).astype(np.float32)
    hu[1] = np.round(hu[1] / 50) * 50          # quantised: many pixels exactly on thresholds
    _check_vs_oracle(hu, min_size=24, border_margin=8)


def test_masks_random_component_soup():
    """Union-find stress: random HU noise gives thousands of small components, long snakes
    and nested holes."""
    rng = np.random.default_rng(5)
    base = rng.choice(np.array([-1024, -800, -300, 40, 250, 700], np.float32), size=(3, 128, 128),
                      p=[0.1, 0.35, 0.05, 0.3, 0.1, 0.1])
    _check_vs_oracle(base, min_size=4, border_margin=2)


def test_hu_transform_matches_reference_golden(golden_dir):
    z, raw, slope, inter = _golden(golden_dir, "hu_64")
    r, s, i = (torch.from_numpy(x).to(DEV) for x in (raw, slope, inter))
    for tag, lo, hi in (("soft", -150, 250), ("lung", -1000, -150)):
        for sq in (True, False):
            hu, img = ops.hu_transform(r, s, i, lo, hi, soft=sq)
            want = z[f"{tag}_{'sq' if sq else 'lin'}"]
            # linear branch: bit-exact; soft branch: expf vs numpy's float32 exp (<= 1 ulp)
            tol = 0 if not sq else 2e-7
            np.testing.assert_allclose(img.cpu().numpy(), want, rtol=0, atol=tol)
            np.testing.assert_array_equal(hu.cpu().numpy(), raw.astype(np.float32) * slope[:, None, None]
                                          + inter[:, None, None])


def test_hu_transform_full_size_vs_oracle():
    raw, slope, inter = phantom.ct_batch(51, 4, 512)
    r, s, i = (torch.from_numpy(x).to(DEV) for x in (raw, slope, inter))
    _, img = ops.hu_transform(r, s, i, -1000, -150, soft=True)
    img = img.cpu().numpy()
    for n in range(4):
        _, want = masks_ref.hu_transform(raw[n], slope[n], inter[n], -1000, -150, True)
        np.testing.assert_allclose(img[n], want, rtol=0, atol=2e-7)


def test_masks_reject_host_tensors():
    with pytest.raises(RuntimeError):
        ops.anatomical_masks(torch.zeros(1, 8, 8), ["lung"])
