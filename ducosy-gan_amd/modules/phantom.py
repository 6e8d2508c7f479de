"""Synthetic chest-CT slices for the input pipeline (no patient data is available offline).

Each slice is a stored-pixel int16 image with a per-slice RescaleSlope / RescaleIntercept, as a
DICOM slice hands it to modules/dataset.py:114-120 of the reference.  The anatomy is drawn so
that every branch of modules/mask_generator.py fires: two lungs with vessels inside them
(lung-mask holes), low-density specks below the component-size limit, a contrast-filled aorta
inside the lung hull (a bone candidate that the mediastinal exclusion removes), a spine with a
hollow body (bone hole filling) and a bar that reaches from the spine into the hull (region
growing brings it back), ribs and a sternum outside the hull, plus slices where the two-lung
gate fails (one lung, tiny lungs, empty air) and slices with HU values exactly on every
threshold.  Deterministic in (seed, index, size): numpy PCG64.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

KINDS = ("chest", "one_lung", "air", "tiny_lungs", "edges")


def _disc(u, v, cy, cx, ry, rx=None):
    rx = ry if rx is None else rx
    return ((u - cy) / ry) ** 2 + ((v - cx) / rx) ** 2 <= 1.0


def slice_hu(seed: int, index: int, size: int = 512, kind: str = None) -> np.ndarray:
    """One synthetic slice in HU (float64, before storage quantisation)."""
    rng = np.random.default_rng([seed, index, size])
    kind = kind or KINDS[index % len(KINDS)]
    S = size
    u, v = np.mgrid[0:S, 0:S].astype(np.float64)
    u = (u + 0.5) / S
    v = (v + 0.5) / S
    j = lambda s=0.02: rng.uniform(-s, s)
    hu = -1024.0 + rng.normal(0, 3, (S, S))
    if kind == "air":
        return hu
    cy, cx = 0.5 + j(), 0.5 + j()
    ay, ax = 0.40 + j(), 0.45 + j()
    body = _disc(u, v, cy, cx, ay, ax)
    hu[body] = -100 + rng.normal(0, 15, body.sum())                       # subcutaneous fat
    inner = _disc(u, v, cy, cx, 0.9 * ay, 0.9 * ax)
    hu[inner] = 40 + rng.normal(0, 15, inner.sum())                       # soft tissue
    lungs = [(0.45 + j(), 0.30 + j(), 0.20 + j(), 0.12 + j(0.01)),
             (0.45 + j(), 0.70 + j(), 0.20 + j(), 0.12 + j(0.01))]
    if kind == "one_lung":
        lungs = lungs[:1]
    if kind == "tiny_lungs":
        lungs = [(ly, lx, 0.035, 0.03) for ly, lx, _, _ in lungs]
    lung_any = np.zeros((S, S), bool)
    for ly, lx, ry, rx in lungs:
        m = _disc(u, v, ly, lx, ry, rx)
        lung_any |= m
        hu[m] = -850 + rng.normal(0, 40, m.sum())
        for _ in range(6):                                                 # vessels (holes)
            a, r = rng.uniform(0, 2 * np.pi), rng.uniform(0.0, 0.7)
            vy, vx = ly + r * ry * np.sin(a), lx + r * rx * np.cos(a)
            vm = _disc(u, v, vy, vx, rng.uniform(0.006, 0.012))
            hu[vm] = 80 + rng.normal(0, 20, vm.sum())
    heart = _disc(u, v, 0.56, 0.5, 0.12, 0.10)
    hu[heart & ~lung_any] = 45 + rng.normal(0, 10, (heart & ~lung_any).sum())
    aorta = _disc(u, v, 0.40, 0.53, 0.03)
    hu[aorta] = 320 + rng.normal(0, 10, aorta.sum())                       # contrast: bone candidate
    spine = _disc(u, v, 0.80, 0.5, 0.05)
    hu[spine] = 700 + rng.normal(0, 30, spine.sum())
    canc = _disc(u, v, 0.80, 0.5, 0.03)
    hu[canc] = 150 + rng.normal(0, 10, canc.sum())                         # bone hole
    bar = (u > 0.60) & (u < 0.80) & (np.abs(v - 0.5) < 0.012)
    hu[bar] = 450 + rng.normal(0, 10, bar.sum())                           # grows back from the spine
    for a in np.linspace(0.2 * np.pi, 1.8 * np.pi, 10):                  # ribs along the wall
        rr = _disc(u, v, cy - 0.88 * ay * np.cos(a), cx + 0.88 * ax * np.sin(a), 0.012)
        hu[rr] = 600 + rng.normal(0, 20, rr.sum())
    st = _disc(u, v, cy - 0.85 * ay, 0.5, 0.02)
    hu[st] = 500 + rng.normal(0, 20, st.sum())                             # sternum
    for _ in range(5):                                                     # sub-threshold specks
        sm = _disc(u, v, rng.uniform(0.25, 0.75), rng.uniform(0.25, 0.75), 0.005)
        hu[sm & ~lung_any] = -500
    near_edge = (u < 0.05) & (np.abs(v - 0.5) < 0.05) & body
    hu[near_edge] = -400                                                   # inside the border margin
    if kind == "edges":
        # exact threshold values: lung rims at -300 (hull vertices), vessel/mediastinum/bone limits
        for ly, lx, ry, rx in lungs:
            m = _disc(u, v, ly, lx, ry, rx)
            rows = np.where(m.any(1))[0]
            for r in rows:
                cols = np.where(m[r])[0]
                hu[r, cols[0]] = -300
                hu[r, cols[-1]] = -300
        pick = rng.uniform(size=(S, S))
        hu[(pick < 0.01) & lung_any] = -300
        hu[(pick > 0.99) & heart] = 450
        hu[(pick > 0.98) & (pick <= 0.99) & heart] = 200
        hu[(pick > 0.97) & (pick <= 0.98) & lung_any] = 600
        hu[(pick < 0.005) & ~body] = -1000
    return hu


def ct_batch(seed: int, n: int, size: int = 512, kinds=None) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(raw int16 [n,H,W], slope float32 [n], intercept float32 [n]): stored pixel values with a
    per-slice rescale (slope 1 or 0.5, intercept -1024 or -1000), as pixel_array gives them."""
    raws, slopes, inters = [], [], []
    for i in range(n):
        hu = slice_hu(seed, i, size, None if kinds is None else kinds[i % len(kinds)])
        slope, inter = (1.0, -1024.0) if i % 3 else (0.5, -1000.0)
        raw = np.clip(np.round((hu - inter) / slope), -32768, 32767).astype(np.int16)
        raws.append(raw)
        slopes.append(slope)
        inters.append(inter)
    return np.stack(raws), np.array(slopes, np.float32), np.array(inters, np.float32)
