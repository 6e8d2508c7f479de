"""CPU restatement of the reference's input pipeline: HU transform + anatomical masks.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import anything under ``oracle/``.

Follows, per 2-D slice (the way modules/dataset.py:114-132 calls it):
  * preprocess.apply_hu_transform / apply_soft_squeezing   modules/preprocess.py:6-55
  * mask_generator.detect_lung                              modules/mask_generator.py:11-36
  * mask_generator.detect_lung_vessels (2-D branch)         modules/mask_generator.py:55-76
  * mask_generator.detect_mediastinum (2-D branch)          modules/mask_generator.py:102-138
  * mask_generator.detect_bone (2-D branch)                 modules/mask_generator.py:177-245
  * mask_generator.generate_anatomical_masks                modules/mask_generator.py:313-347
Third-party pieces the reference calls, restated or reused:
  * scipy.ndimage.label / binary_fill_holes (default cross structure = 4-connectivity): used
    directly (scipy 1.15 here; the reference's requirements leave it unpinned);
  * scipy.spatial.ConvexHull (qhull): used directly for the vertex set and order;
  * matplotlib.path.Path.contains_points (matplotlib _path.h point_in_path, radius 0):
    restated below as the division-free crossing-number rule; pinned against the reference
    itself (with matplotlib 3.10) by tests/golden/masks_*.npz.
"""
from __future__ import annotations

import numpy as np
from scipy import ndimage
from scipy.spatial import ConvexHull

MASK_KINDS = ("lung", "mediastinum", "bone", "lung_vessel")


def hu_transform(raw, slope, intercept, hu_min, hu_max, soft=True, sigma=50):
    """preprocess.py:43-55 (+ apply_soft_squeezing :6-40) in numpy float32, one slice."""
    image = raw.astype(np.float32)
    image = image * float(slope) + float(intercept)
    hu = image.copy()
    image = np.clip(image, hu_min, hu_max)
    if soft:
        normalized = (image - hu_min) / (hu_max - hu_min)
        k = 10.0 / sigma
        s = 1.0 / (1.0 + np.exp(-k * (normalized - 0.9)))
        r = np.where(normalized < 0.9, normalized, 0.9 + (1.0 - 0.9) * s)
        image = 2.0 * r - 1.0
    else:
        image = 2 * (image - hu_min) / (hu_max - hu_min) - 1
    return hu, image.astype(np.float32)


def points_in_polygon(vertices: np.ndarray, H: int, W: int) -> np.ndarray:
    """matplotlib Path(vertices).contains_points over the (row, col) grid: crossing number with
    the edge test ((vy1 - ty)(vx0 - vx1) >= (vx1 - tx)(vy0 - vy1)) == (vy1 >= ty), the polygon
    implicitly closed (point_in_path in matplotlib's _path.h).  x = row, y = col."""
    tx, ty = np.mgrid[0:H, 0:W]
    tx = tx.astype(np.int64)
    ty = ty.astype(np.int64)
    inside = np.zeros((H, W), bool)
    v = vertices.astype(np.int64)
    n = len(v)
    for j in range(n):
        x0, y0 = v[j - 1]
        x1, y1 = v[j]
        f0 = y0 >= ty
        f1 = y1 >= ty
        hit = (f0 != f1) & ((((y1 - ty) * (x0 - x1)) >= ((x1 - tx) * (y0 - y1))) == f1)
        inside ^= hit
    return inside


def _lung_gate(lung, body):
    """>= 2 lung regions and lung/body area >= 0.1 (mask_generator.py:64-68 / 112-116 / 192-196)."""
    _, nreg = ndimage.label(lung)
    body_area, lung_area = int(body.sum()), int(lung.sum())
    return nreg >= 2 and body_area > 0 and (lung_area / body_area) >= 0.1


def _hull_inside(lung):
    """(inside mask, ok): convex hull of the lung pixels rasterised by the crossing rule; ok is
    False where the reference takes its fallback (< 3 pixels, or qhull fails on collinear)."""
    coords = np.argwhere(lung == 1)
    if len(coords) < 3:
        return lung.astype(bool), False
    try:
        hull = ConvexHull(coords)
    except Exception:  # qhull raises on flat input; the reference's bare except (:127, :221)
        return lung.astype(bool), False
    return points_in_polygon(coords[hull.vertices], *lung.shape), True


def masks_2d(hu, mask_types=MASK_KINDS, lung_lower=-1000, lung_upper=-300, min_size=64, border_margin=32,
             vessel_lower=-300, vessel_upper=600, mediastinum_lower=-300, mediastinum_upper=450,
             bone_threshold=200, spine_margin_ratio=0.25):
    """generate_anatomical_masks on one 2-D HU slice -> {name: uint8 mask}."""
    H, W = hu.shape
    body = hu > -1000
    # detect_lung
    lung = ((hu >= lung_lower) & (hu <= lung_upper) & body).astype(np.uint8)
    lung[:border_margin, :] = 0
    lung[H - border_margin:, :] = 0
    lung[:, :border_margin] = 0
    lung[:, W - border_margin:] = 0
    lab, nf = ndimage.label(lung)
    if nf:
        sizes = np.bincount(lab.ravel(), minlength=nf + 1)
        small = sizes < min_size
        small[0] = False
        lung[small[lab]] = 0
    gate = _lung_gate(lung, body)
    out = {}
    if "lung" in mask_types:
        out["lung"] = lung
    inside, ok = _hull_inside(lung) if gate else (None, False)
    if "mediastinum" in mask_types:
        if gate:
            cand = inside != lung.astype(bool)        # uint8 `convex_hull - lung` is nonzero
            hu_ok = (hu >= mediastinum_lower) & (hu <= mediastinum_upper)
            out["mediastinum"] = (cand & hu_ok).astype(np.uint8)
        else:
            out["mediastinum"] = np.zeros_like(lung)
    if "bone" in mask_types:
        all_bone = (hu >= bone_threshold) & body
        bone = all_bone.copy()
        if gate and ok:
            spine = np.zeros((H, W), bool)
            spine[int(H * (1 - spine_margin_ratio)):, :] = True
            bone &= ~(inside & ~lung.astype(bool) & ~spine)
        if (all_bone & ~bone).any():                  # region growing (:224-239)
            lab, _ = ndimage.label(all_bone)
            keep = np.zeros(lab.max() + 1, bool)
            keep[np.unique(lab[bone])] = True
            keep[0] = False
            bone |= keep[lab] & (hu >= bone_threshold)
        if bone.any():
            bone = ndimage.binary_fill_holes(bone)
        out["bone"] = bone.astype(np.uint8)
    if "lung_vessel" in mask_types:
        if gate:
            filled = ndimage.binary_fill_holes(lung)
            cand = filled & ~lung.astype(bool)
            out["lung_vessel"] = (cand & (hu >= vessel_lower) & (hu <= vessel_upper)).astype(np.uint8)
        else:
            out["lung_vessel"] = np.zeros_like(lung)
    return out


def masks_batch(hu, mask_types, **params):
    """[N,H,W] HU -> float32 [N, len(mask_types), H, W] in mask_types order (dataset.py:135-158)."""
    out = np.zeros((hu.shape[0], len(mask_types)) + hu.shape[1:], np.float32)
    for n in range(hu.shape[0]):
        m = masks_2d(hu[n], mask_types, **params)
        for c, k in enumerate(mask_types):
            out[n, c] = m[k]
    return out
