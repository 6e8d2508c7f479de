"""Drop-in for the reference's modules/postprocess.py (volume post-processing of generate.py).

Same functions, signatures, defaults and results as modules/postprocess.py:6-301
(``postprocess_ct_volume``, ``unsharp_mask``, ``adaptive_smooth``, ``apply_kalman_filter``,
``kalman_filter_1d``, ``apply_diffmap``); this is the host side of generate.py's synthesis
stage (generate.py:16, 246-254), after the GPU Generator passes.  Where the reference loops
over pixels in Python (the 'interpolation' and 'kalman' methods, postprocess.py:78-93 and
:217-230) the same per-pixel arithmetic runs vectorised over the whole slice plane:

* 'interpolation': one not-a-knot cubic B-spline through every z column at once
  (scipy.interpolate.make_interp_spline along axis 0, which is what interp1d(kind='cubic')
  builds per column), evaluated at the reference's 2x grid and subsampled back;
* 'kalman': the gain sequence of the scalar filter depends only on the two variances, so the
  state update runs for all pixels in lock-step, in float64 as the reference.

Checked against outputs of the reference module itself (tests/golden/make_golden_post.py,
tests/test_cpu_postprocess.py).
"""
from __future__ import annotations

import numpy as np
from scipy.interpolate import make_interp_spline
from scipy.ndimage import gaussian_filter, gaussian_filter1d, median_filter

METHODS = ("gaussian", "gaussian3d", "adaptive", "median", "interpolation", "kalman")


def postprocess_ct_volume(volume, method="gaussian3d", enhance_sharpness=True, hu_threshold=750, **kwargs):
    """Smooth a [slices, H, W] CT volume along z (and optionally sharpen in-plane), keep the
    voxels at or above ``hu_threshold`` (bone) unchanged, return int16 (postprocess.py:6-112).

    method: 'gaussian' (sigma=1.0, z only), 'gaussian3d' (sigma_z=2.0, sigma_xy=0.5),
    'adaptive' (base_sigma=1.5, max_sigma=3.0), 'median' (kernel_size=3, z only),
    'interpolation' (cubic spline in z), 'kalman' (process_variance=1e-5,
    measurement_variance=1e-2); sharpening: sharpen_amount=0.5, sharpen_radius=1.0."""
    vol = np.asarray(volume)
    original = vol.copy()
    keep = vol >= hu_threshold
    if method == "gaussian":
        out = gaussian_filter1d(vol, sigma=kwargs.get("sigma", 1.0), axis=0)
    elif method == "gaussian3d":
        sxy = kwargs.get("sigma_xy", 0.5)
        out = gaussian_filter(vol, sigma=(kwargs.get("sigma_z", 2.0), sxy, sxy))
    elif method == "adaptive":
        out = adaptive_smooth(vol, kwargs.get("base_sigma", 1.5), kwargs.get("max_sigma", 3.0))
    elif method == "median":
        out = median_filter(vol, size=(kwargs.get("kernel_size", 3), 1, 1))
    elif method == "interpolation":
        n = vol.shape[0]
        spline = make_interp_spline(np.arange(n), vol, k=3, axis=0)
        fine = spline(np.linspace(0, n - 1, 2 * n))
        out = fine[::2].astype(vol.dtype)  # the reference fills a zeros(vol.dtype) array
    elif method == "kalman":
        out = apply_kalman_filter(vol, kwargs.get("process_variance", 1e-5),
                                  kwargs.get("measurement_variance", 1e-2))
    else:
        raise ValueError(f"Unknown method: {method}. Choose from 'gaussian', 'gaussian3d', 'adaptive', 'median', "
                         "'interpolation', 'kalman'")
    if enhance_sharpness:
        out = unsharp_mask(out, original, amount=kwargs.get("sharpen_amount", 0.5),
                           radius=kwargs.get("sharpen_radius", 1.0))
    out[keep] = original[keep]
    return out.astype(np.int16)


def unsharp_mask(smoothed_volume, original_volume, amount=0.5, radius=1.0):
    """In-plane unsharp masking of the smoothed volume with a blend of its own and the
    original's high frequencies, clipped to the original's range (postprocess.py:114-160)."""
    sm = np.asarray(smoothed_volume).astype(np.float64)
    og = np.asarray(original_volume).astype(np.float64)
    blur = (0, radius, radius)
    detail = (1 - amount) * (sm - gaussian_filter(sm, sigma=blur)) + amount * (og - gaussian_filter(og, sigma=blur))
    return np.clip(sm + detail * amount, og.min(), og.max())


def adaptive_smooth(volume, base_sigma=1.5, max_sigma=3.0):
    """postprocess.py:163-201: z Gaussian (base_sigma) then a (max_sigma, 0.3, 0.3) 3-D
    Gaussian, in float64.  (The reference also measures the inter-slice differences but never
    uses them; they have no effect on the result.)"""
    out = np.asarray(volume).astype(np.float64)
    out = gaussian_filter1d(out, sigma=base_sigma, axis=0)
    return gaussian_filter(out, sigma=(max_sigma, 0.3, 0.3))


def apply_kalman_filter(volume, process_variance=1e-5, measurement_variance=1e-2):
    """postprocess.py:204-232: the 1-D Kalman filter of kalman_filter_1d along z for every
    pixel (float64)."""
    vol = np.asarray(volume)
    z = vol.reshape(vol.shape[0], -1).astype(np.float64)
    return _kalman_columns(z, process_variance, measurement_variance).reshape(vol.shape)


def kalman_filter_1d(measurements, process_variance, measurement_variance):
    """postprocess.py:235-272: scalar Kalman filter of one series (initial state = first
    measurement, initial covariance 1)."""
    m = np.asarray(measurements, dtype=np.float64)
    return _kalman_columns(m[:, None], process_variance, measurement_variance)[:, 0]


def _kalman_columns(z, q, r):
    """z: [n, cols] float64 -> filtered [n, cols]; every column runs the same gain sequence."""
    out = np.empty_like(z)
    x = z[0].copy()
    p = 1.0
    for k in range(z.shape[0]):
        pp = p + q
        gain = pp / (pp + r)
        x = x + gain * (z[k] - x)
        p = (1 - gain) * pp
        out[k] = x
    return out


def apply_diffmap(volume, diff_volume, threshold=8):
    """postprocess.py:275-301: add a difference map (values below ``threshold`` zeroed, then
    cast to uint8) to the volume.  Like the reference, an ndarray ``diff_volume`` is thresholded
    in place."""
    vol = volume if isinstance(volume, np.ndarray) else np.array(volume)
    diff = diff_volume if isinstance(diff_volume, np.ndarray) else np.array(diff_volume)
    diff[diff < threshold] = 0
    return vol + diff.astype(np.uint8)
