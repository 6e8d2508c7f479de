"""Input-pipeline oracle (oracle/masks_ref.py) pinned against the reference's own outputs
(tests/golden/masks_*.npz, hu_64.npz written by make_golden_masks.py from the reference's
modules/mask_generator.py and modules/preprocess.py), plus the synthetic-slice generator."""
import zlib

import numpy as np
import pytest

from modules import phantom
from oracle import masks_ref

KINDS = ("lung", "mediastinum", "bone", "lung_vessel")


def _golden(golden_dir, name):
    z = np.load(f"{golden_dir}/{name}.npz")
    n, S = int(z["n"]), int(z["size"])
    raw, slope, inter = phantom.ct_batch(int(z["seed"]), n, S)
    assert np.uint32(zlib.crc32(raw.tobytes())) == z["crc"], "phantom drifted from the fixture inputs"
    return z, raw, slope, inter


def unpack(z, i, c):
    S = int(z["size"])
    return np.unpackbits(z["packed"][i, c])[:S * S].reshape(S, S)


@pytest.mark.parametrize("name", ["masks_128", "masks_512"])
def test_oracle_masks_match_reference(golden_dir, name):
    z, raw, slope, inter = _golden(golden_dir, name)
    kw = dict(min_size=int(z["min_size"]), border_margin=int(z["border"]))
    for i in range(raw.shape[0]):
        hu = raw[i].astype(np.float32) * float(slope[i]) + float(inter[i])
        m = masks_ref.masks_2d(hu, KINDS, **kw)
        for c, k in enumerate(KINDS):
            np.testing.assert_array_equal(m[k], unpack(z, i, c), err_msg=f"slice {i} {k}")


def test_golden_slices_cover_every_branch(golden_dir):
    """The fixture slices exercise the two-lung gate both ways, vessels, mediastinum, bone."""
    z, raw, _, _ = _golden(golden_dir, "masks_512")
    sums = np.array([[unpack(z, i, c).sum() for c in range(4)] for i in range(raw.shape[0])])
    assert (sums[:, 1] > 0).any() and (sums[:, 1] == 0).any()       # mediastinum gated
    assert (sums[:, 3] > 0).any()                                   # lung vessels present
    assert (sums[:, 2] > 0).sum() >= 3                              # bone on every body slice
    assert (sums.sum(1) == 0).any()                                 # an empty (air) slice


def test_oracle_hu_transform_matches_reference(golden_dir):
    z, raw, slope, inter = _golden(golden_dir, "hu_64")
    for tag, lo, hi in (("soft", -150, 250), ("lung", -1000, -150)):
        for sq in (True, False):
            want = z[f"{tag}_{'sq' if sq else 'lin'}"]
            for i in range(raw.shape[0]):
                _, img = masks_ref.hu_transform(raw[i], slope[i], inter[i], lo, hi, sq)
                np.testing.assert_array_equal(img, want[i])


def test_crossing_rule_on_a_square():
    """Boundary convention of matplotlib's point_in_path for a CCW unit-grid square."""
    sq = np.array([[1, 1], [3, 1], [3, 3], [1, 3]])
    inside = masks_ref.points_in_polygon(sq, 5, 5)
    # interior point, and the half-open edges of the crossing rule
    assert inside[2, 2]
    assert not inside[0, 0] and not inside[4, 4]
    assert inside.sum() == len(np.argwhere(inside))
