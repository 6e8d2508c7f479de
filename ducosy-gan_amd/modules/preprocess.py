"""Drop-in for the reference's modules/preprocess.py on the MI355X kernels.

Same functions and arguments (modules/preprocess.py:6-113).  apply_soft_squeezing and
apply_hu_transform run dcs_hu_transform on the GPU (float32 op order of the numpy original;
tests/test_gpu_masks.py) and hand numpy arrays back where the reference does;
apply_windowing / postprocess_tensor are the reference's small tensor/array maps (display and
DICOM write-back, not on the training step).  DICOM files are read with modules/dicom.py
(pydicom is not installed in this image).
"""
from __future__ import annotations

import numpy as np
import torch

from .hip import ops


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("the HU transform runs on the MI355X kernels; no GPU is visible")
    return torch.device("cuda", torch.cuda.current_device())


def _transform(pixels, slope, intercept, hu_min, hu_max, soft, sigma=50):
    is_np = not isinstance(pixels, torch.Tensor)
    t = torch.from_numpy(np.ascontiguousarray(pixels)) if is_np else pixels
    two_d = t.dim() == 2
    t = t[None] if two_d else t
    dev = t.device if t.is_cuda else _device()
    if t.dtype not in (torch.int16, torch.float32) and not (hasattr(torch, "uint16") and t.dtype == torch.uint16):
        t = t.to(torch.float32)
    t = t.to(dev)
    n = t.shape[0]
    s = torch.full((n,), float(slope), device=dev)
    b = torch.full((n,), float(intercept), device=dev)
    _, img = ops.hu_transform(t, s, b, hu_min, hu_max, soft=soft, sigma=sigma, want_hu=False)
    img = img[0] if two_d else img
    return img.cpu().numpy() if is_np else img


def apply_soft_squeezing(image, hu_min, hu_max, sigma=50):
    """preprocess.py:6-40 on HU values already clipped to [hu_min, hu_max] (as the reference
    calls it, :47-50; clipping again is the identity there)."""
    if isinstance(image, np.ndarray):
        image = image.astype(np.float32)
    return _transform(image, 1.0, 0.0, hu_min, hu_max, True, sigma)


def apply_hu_transform(dicom_img, hu_min, hu_max, use_soft_squeezing=True):
    """preprocess.py:43-55: stored pixels -> HU -> clip -> soft squeeze / linear -> [-1, 1]."""
    return _transform(dicom_img.pixel_array, float(dicom_img.RescaleSlope), float(dicom_img.RescaleIntercept),
                      hu_min, hu_max, use_soft_squeezing)


def apply_windowing(tensor_img, args):
    """preprocess.py:58-65 (display windowing of a model output)."""
    hu_img = (tensor_img + 1.0) / 2.0 * (args.hu_max - args.hu_min) + args.hu_min
    wc, ww = args.window_center, args.window_width
    lo, hi = wc - ww / 2.0, wc + ww / 2.0
    return (torch.clamp(hu_img, lo, hi) - lo) / ww


def preprocess_dicom(dcm_path, soft_tissue_hu_min, soft_tissue_hu_max, lung_hu_min, lung_hu_max):
    """preprocess.py:68-90: (soft-tissue [1,H,W], lung [1,H,W], dataset), linear [-1, 1]."""
    from .dicom import dcmread
    dcm = dcmread(dcm_path)
    slope, inter = float(dcm.RescaleSlope), float(dcm.RescaleIntercept)
    soft = _transform(dcm.pixel_array, slope, inter, soft_tissue_hu_min, soft_tissue_hu_max, False)
    lung = _transform(dcm.pixel_array, slope, inter, lung_hu_min, lung_hu_max, False)
    return torch.from_numpy(soft).unsqueeze(0), torch.from_numpy(lung).unsqueeze(0), dcm


def postprocess_tensor(output_tensor, original_dcm, hu_min, hu_max):
    """preprocess.py:93-113: model output in [-1, 1] -> stored values of the original dtype."""
    out = output_tensor.detach().cpu().squeeze().numpy()
    hu = (out + 1.0) / 2.0 * (hu_max - hu_min) + hu_min
    px = (hu - float(original_dcm.RescaleIntercept)) / float(original_dcm.RescaleSlope)
    return px.astype(original_dcm.pixel_array.dtype)
