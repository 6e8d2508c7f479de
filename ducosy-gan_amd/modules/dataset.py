"""Drop-in for the reference's modules/dataset.py with the per-slice work moved to the GPU.

The reference's DicomDataset.__getitem__ (modules/dataset.py:109-181) does everything per
slice on a CPU worker: DICOM decode, HU transform with soft squeezing, scipy/matplotlib mask
generation (~65 ms per 512x512 slice in the reference here), ToTensor + Resize.  Here:

  * DicomDataset keeps the reference's constructor, file pairing and slice ordering
    (:63-104: NCCT/CECT folders, InstanceNumber -> SliceLocation -> filename sort, mask
    files named like the NCCT slice) and its __getitem__ only decodes the files (stored int16
    pixels + rescale per slice, and mask files when masks are not auto-generated);
  * SliceBatchPreprocessor turns a collated batch into the reference's batch
    {"A": [N,1,S,S], "B": [N,1,S,S], "masks": [N,m,S,S]} on the GPU in one pass:
    dcs_hu_transform for both domains, dcs_anatomical_masks on the NCCT HU in mask_types
    order, and the Resize of the transform when the slice size differs from img_size
    (bilinear antialias for images and mask files, nearest for generated masks, :141-150).

DICOM files are read with modules/dicom.py (pydicom is not installed in this image).
"""
from __future__ import annotations

import glob
import os
from typing import List

import numpy as np
import torch
import torch.nn.functional as F

from . import dicom
from .hip import ops


def load_mask_from_dicom(mask_path):
    """dataset.py:16-28: binary float32 mask from a mask DICOM, None when missing/unreadable."""
    if not os.path.exists(mask_path):
        return None
    try:
        return (dicom.dcmread(mask_path).pixel_array > 0).astype(np.float32)
    except Exception as e:  # the reference warns and continues
        print(f"Warning: Failed to load mask from {mask_path}: {e}")
        return None


def _sort_slices(files: List[str]) -> List[str]:
    """dataset.py:81-90: InstanceNumber, else SliceLocation, else filename order."""
    try:
        return sorted(files, key=lambda x: int(dicom.dcmread(x, stop_before_pixels=True).InstanceNumber))
    except (AttributeError, KeyError, ValueError):
        try:
            return sorted(files, key=lambda x: float(dicom.dcmread(x, stop_before_pixels=True).SliceLocation))
        except (AttributeError, KeyError, ValueError):
            print("Warning: InstanceNumber/SliceLocation not found. Falling back to filename sort.")
            return files


class DicomDataset(torch.utils.data.Dataset):
    """modules/dataset.py:61-107; items are decoded slices, see SliceBatchPreprocessor."""

    def __init__(self, patient_dirs, args, transform=None):
        self.args = args
        self.transform = transform  # kept for API parity; the resize runs in SliceBatchPreprocessor
        self.paired_files = []
        self.use_masks = getattr(args, "use_masks", False)
        self.auto_generate_masks = getattr(args, "auto_generate_masks", False)
        self.mask_types = getattr(args, "mask_types", ["lung", "mediastinum", "bone", "lung_vessel"])
        self.mask_folders = getattr(args, "mask_folders", [])
        for patient_dir in patient_dirs:
            ncct = sorted(glob.glob(os.path.join(patient_dir, args.ncct_folder, "*.dcm")))
            cect = sorted(glob.glob(os.path.join(patient_dir, args.cect_folder, "*.dcm")))
            if not ncct or not cect:
                continue
            ncct, cect = _sort_slices(ncct), _sort_slices(cect)
            for a, b in zip(ncct, cect):
                mask_paths = {}
                if self.use_masks and not self.auto_generate_masks:
                    for name in self.mask_folders:
                        p = os.path.join(patient_dir, name, os.path.basename(a))
                        if os.path.exists(p):
                            mask_paths[name] = p
                self.paired_files.append((a, b, mask_paths))

    def __len__(self):
        return len(self.paired_files)

    def __getitem__(self, index):
        a_path, b_path, mask_paths = self.paired_files[index]
        a, b = dicom.dcmread(a_path), dicom.dcmread(b_path)
        item = {"A_raw": torch.from_numpy(a.pixel_array.astype(np.int16)),
                "B_raw": torch.from_numpy(b.pixel_array.astype(np.int16)),
                "A_rescale": torch.tensor([float(a.RescaleSlope), float(a.RescaleIntercept)]),
                "B_rescale": torch.tensor([float(b.RescaleSlope), float(b.RescaleIntercept)])}
        if self.use_masks and not self.auto_generate_masks and mask_paths:
            H, W = item["A_raw"].shape
            ms = []
            for name in self.mask_folders:
                m = load_mask_from_dicom(mask_paths[name]) if name in mask_paths else None
                ms.append(torch.from_numpy(m) if m is not None else torch.full((H, W), float("nan")))
            item["mask_files"] = torch.stack(ms)  # NaN plane = missing -> zeros after resize
        return item


def collate(samples):
    """Stack equally-sized slices; a list of per-slice batches when sizes differ."""
    shapes = {tuple(s["A_raw"].shape) for s in samples}
    keys = set.intersection(*(set(s) for s in samples))
    if len(shapes) == 1:
        return {k: torch.stack([s[k] for s in samples]) for k in keys}
    return [{k: s[k][None] for k in keys} for s in samples]


class SliceBatchPreprocessor:
    """Decoded slices -> the reference's training batch, on the device (see module doc)."""

    def __init__(self, args, device):
        self.args = args
        self.device = torch.device(device)
        self.size = int(args.img_size)
        self.soft = bool(getattr(args, "use_soft_squeezing", True))
        self.use_masks = bool(getattr(args, "use_masks", False))
        self.auto = bool(getattr(args, "auto_generate_masks", False))
        self.mask_types = list(getattr(args, "mask_types", []))

    def _resize(self, x, mode):
        if tuple(x.shape[-2:]) == (self.size, self.size):
            return x
        if mode == "nearest":
            return F.interpolate(x, size=(self.size, self.size), mode="nearest")
        return F.interpolate(x, size=(self.size, self.size), mode="bilinear", align_corners=False, antialias=True)

    def _one(self, batch):
        dev = self.device
        ra, rb = batch["A_raw"].to(dev, non_blocking=True), batch["B_raw"].to(dev, non_blocking=True)
        sa, sb = batch["A_rescale"].to(dev), batch["B_rescale"].to(dev)
        hu_a, img_a = ops.hu_transform(ra, sa[:, 0], sa[:, 1], self.args.hu_min, self.args.hu_max, soft=self.soft)
        _, img_b = ops.hu_transform(rb, sb[:, 0], sb[:, 1], self.args.hu_min, self.args.hu_max, soft=self.soft,
                                    want_hu=False)
        out = {"A": self._resize(img_a[:, None], "bilinear"), "B": self._resize(img_b[:, None], "bilinear")}
        if self.use_masks and self.auto and self.mask_types:
            known = [k for k in self.mask_types if k in ops.MASK_KINDS]
            m = ops.anatomical_masks(hu_a, known) if known else None
            chans = []
            for k in self.mask_types:  # unknown kinds -> zero planes (dataset.py:152-154)
                chans.append(m[:, known.index(k)] if k in known else torch.zeros_like(hu_a))
            out["masks"] = self._resize(torch.stack(chans, 1), "nearest")
        elif self.use_masks and "mask_files" in batch:
            mf = batch["mask_files"].to(dev)
            missing = torch.isnan(mf).flatten(2).any(-1)
            mf = self._resize(torch.nan_to_num(mf, nan=0.0), "bilinear")
            out["masks"] = torch.where(missing[..., None, None], torch.zeros_like(mf), mf)
        return out

    def __call__(self, batch):
        if isinstance(batch, list):
            parts = [self._one(b) for b in batch]
            return {k: torch.cat([p[k] for p in parts]) for k in parts[0]}
        return self._one(batch)
