"""Drop-in for the reference's modules/mask_generator.py on the MI355X kernels.

Same functions and arguments (modules/mask_generator.py:11-347): detect_lung,
detect_lung_vessels, detect_mediastinum, detect_bone, generate_anatomical_masks.  Inputs are HU
arrays, 2-D [H,W] or 3-D [Z,H,W] (the reference's 3-D branches are its 2-D rule applied per
slice), as numpy arrays or torch tensors; numpy in -> numpy uint8 out, tensor in -> tensor out
on the tensor's device.  Every call runs dcs_anatomical_masks on the GPU (bit-exact with the
reference, tests/test_gpu_masks.py); there is no CPU path — without a GPU the calls raise.
"""
from __future__ import annotations

import numpy as np
import torch

from .hip import ops


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("mask generation runs on the MI355X kernels; no GPU is visible")
    return torch.device("cuda", torch.cuda.current_device())


def _as_batch(x, dtype):
    """(tensor [Z,H,W] on the GPU, was_numpy, was_2d)."""
    is_np = not isinstance(x, torch.Tensor)
    t = torch.from_numpy(np.ascontiguousarray(x)) if is_np else x
    two_d = t.dim() == 2
    if two_d:
        t = t[None]
    if t.dim() != 3:
        raise ValueError("expected a 2-D slice or a 3-D [Z,H,W] volume")
    if not t.is_cuda:
        t = t.to(_device())
    return t.to(dtype).contiguous(), is_np, two_d


def _run(hu_volume, kind, lung_mask=None, **params):
    hu, is_np, two_d = _as_batch(hu_volume, torch.float32)
    lm = None
    if lung_mask is not None:
        lm, _, _ = _as_batch(lung_mask, torch.uint8)
        if lm.shape != hu.shape:
            raise ValueError("lung_mask must have the HU volume's shape")
    out = ops.anatomical_masks(hu, [kind], lung_mask=lm, **params)[:, 0].to(torch.uint8)
    if two_d:
        out = out[0]
    return out.cpu().numpy() if is_np else out


def detect_lung(hu_volume, lung_lower=-1000, lung_upper=-300, min_size=64, border_margin=32):
    """modules/mask_generator.py:11-52."""
    return _run(hu_volume, "lung", lung_lower=lung_lower, lung_upper=lung_upper, min_size=min_size,
                border_margin=border_margin)


def detect_lung_vessels(hu_volume, lung_mask, vessel_lower=-300, vessel_upper=600):
    """modules/mask_generator.py:55-99."""
    return _run(hu_volume, "lung_vessel", lung_mask, vessel_lower=vessel_lower, vessel_upper=vessel_upper)


def detect_mediastinum(hu_volume, lung_mask, mediastinum_lower=-300, mediastinum_upper=450):
    """modules/mask_generator.py:102-174."""
    return _run(hu_volume, "mediastinum", lung_mask, mediastinum_lower=mediastinum_lower,
                mediastinum_upper=mediastinum_upper)


def detect_bone(hu_volume, lung_mask, bone_threshold=200, spine_margin_ratio=0.25):
    """modules/mask_generator.py:177-310."""
    return _run(hu_volume, "bone", lung_mask, bone_threshold=bone_threshold,
                spine_margin_ratio=spine_margin_ratio)


def generate_anatomical_masks(hu_image, mask_types=("lung", "mediastinum", "bone", "lung_vessel")):
    """modules/mask_generator.py:313-347: {name: mask} for the requested kinds, all computed by
    one fused kernel pass (the lung mask is shared, as in the reference)."""
    kinds = [k for k in ("lung", "mediastinum", "bone", "lung_vessel") if k in mask_types]
    if not kinds:
        return {}
    hu, is_np, two_d = _as_batch(hu_image, torch.float32)
    out = ops.anatomical_masks(hu, kinds).to(torch.uint8)
    res = {}
    for c, k in enumerate(kinds):
        m = out[:, c]
        m = m[0] if two_d else m
        res[k] = m.cpu().numpy() if is_np else m
    return res
