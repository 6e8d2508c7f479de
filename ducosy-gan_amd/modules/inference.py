"""Inference-side math of the reference's generate.py on the MI355X path.

Mirrors the array arithmetic of modules/preprocess.py:68-113 (HU transform, clipping,
[-1, 1] normalisation, inverse mapping to stored pixel values) and generate.py:144-236 (the
complementary HU-range synthesis), and batches the Generator forward over slices (the
reference runs one slice per call, generate.py:108-111).  DICOM parsing stays on the host
(pydicom, imported lazily by generate.py); nothing here needs it, so the math is testable
without it.
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F


def hu_from_stored(pixels: np.ndarray, slope: float, intercept: float) -> np.ndarray:
    """preprocess.py:76-82: stored pixel values -> HU (float32)."""
    return pixels.astype(np.float32) * float(slope) + float(intercept)


def normalise_hu(hu: np.ndarray, hu_min: float, hu_max: float) -> np.ndarray:
    """preprocess.py:84-90: clip to [hu_min, hu_max] and map linearly to [-1, 1]."""
    x = np.clip(hu, hu_min, hu_max)
    return (2 * (x - hu_min) / (hu_max - hu_min) - 1).astype(np.float32)


def stored_from_output(out: np.ndarray, hu_min: float, hu_max: float, slope: float, intercept: float,
                       dtype) -> np.ndarray:
    """preprocess.py:99-113: model output in [-1, 1] -> HU -> stored values of the original
    DICOM dtype (numpy astype truncation toward zero, as the reference)."""
    hu = (out + 1.0) / 2.0 * (hu_max - hu_min) + hu_min
    return ((hu - float(intercept)) / float(slope)).astype(dtype)


def resize(x: torch.Tensor, size: Tuple[int, int]) -> torch.Tensor:
    """torchvision.transforms.Resize(size, antialias=True) on a [N,C,H,W] float tensor
    (generate.py:52, 107-115): bilinear with antialiasing."""
    if tuple(x.shape[-2:]) == tuple(size):
        return x
    return F.interpolate(x, size=size, mode="bilinear", align_corners=False, antialias=True)


@torch.no_grad()
def translate_slices(model, slices: Sequence[np.ndarray], img_size: int, batch: int = 16,
                     device="cuda", cond: Optional[Sequence[np.ndarray]] = None) -> List[np.ndarray]:
    """Run the Generator over normalised slices ([H,W] float32 each, any size) in batches of
    `batch` at img_size x img_size, and resize each output back to its slice's size
    (generate.py:104-116).  ``cond``: per-slice mask channels [m,H,W] for a mask-conditioned
    Generator (resized nearest, concatenated after the image as in trainer.py:451-453).
    Returns [H,W] float32 arrays in [-1, 1]."""
    out: List[np.ndarray] = []
    for i in range(0, len(slices), batch):
        chunk = slices[i:i + batch]
        x = torch.stack([resize(torch.from_numpy(np.ascontiguousarray(s))[None, None], (img_size, img_size))[0]
                         for s in chunk]).to(device)
        if cond is not None:
            m = torch.stack([F.interpolate(torch.as_tensor(np.ascontiguousarray(c))[None].float(),
                                           size=(img_size, img_size), mode="nearest")[0]
                             for c in cond[i:i + batch]]).to(device)
        y = model(x) if cond is None else model(x, m)  # concat fused into the stem gather
        for s, yi in zip(chunk, y):
            out.append(resize(yi[None], tuple(s.shape))[0, 0].float().cpu().numpy())
    return out


def synthesize(raw_stored: np.ndarray, raw_hu: np.ndarray, soft_stored: np.ndarray, lung_stored: np.ndarray,
               soft_range: Tuple[float, float], lung_range: Tuple[float, float]) -> np.ndarray:
    """generate.py:212-236: start from the NCCT stored values and overwrite the pixels whose
    NCCT HU lies in each model's HU range with that model's output (soft tissue first, lung
    second, so lung wins where the ranges touch)."""
    merged = raw_stored.copy()
    soft = (raw_hu >= soft_range[0]) & (raw_hu <= soft_range[1])
    lung = (raw_hu >= lung_range[0]) & (raw_hu <= lung_range[1])
    merged[soft] = soft_stored[soft]
    merged[lung] = lung_stored[lung]
    return merged


def smooth_volume(volume: Iterable[np.ndarray]) -> np.ndarray:
    """generate.py:246-254: z Gaussian (sigma 0.8) of the merged stored-value volume, then
    modules/postprocess.py's 'gaussian3d' (sigma_z 0.7, sigma_xy 0.05) with sharpening (1.7 /
    1.2); voxels >= 750 keep their value; int16 out."""
    from scipy.ndimage import gaussian_filter1d
    from .postprocess import postprocess_ct_volume
    vol = gaussian_filter1d(np.asarray(volume, dtype=np.float32), sigma=0.8, axis=0)
    return postprocess_ct_volume(vol, method="gaussian3d", sigma_z=0.7, sigma_xy=0.05, enhance_sharpness=True,
                                 sharpen_amount=1.7, sharpen_radius=1.2)
