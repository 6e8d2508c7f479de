"""DICOM I/O (modules/dicom.py, the pydicom-free reader/writer) and the dataset's file pairing
and slice ordering (modules/dataset.py mirroring the reference's dataset.py:63-104), on CPU."""
import copy
import os
import struct

import numpy as np
import pytest
import torch

from modules import dicom, phantom
from modules.dataset import DicomDataset, collate


def _write_tree(root, patients=2, slices=3, size=32, shuffle_instances=True, mask_folders=()):
    raw, slope, inter = phantom.ct_batch(3, patients * slices, size)
    for p in range(patients):
        for name in ("POST VUE", "POST STD"):
            os.makedirs(os.path.join(root, f"P{p}", name), exist_ok=True)
        for m in mask_folders:
            os.makedirs(os.path.join(root, f"P{p}", m), exist_ok=True)
        for s in range(slices):
            k = p * slices + s
            inst = (slices - s) if shuffle_instances else s + 1   # file order != instance order
            for name, off in (("POST VUE", 0), ("POST STD", 7)):
                ds = dicom.new_ct_slice((raw[k] + off).astype(np.int16), float(slope[k]), float(inter[k]),
                                        instance=inst, uid_suffix=f"{p}.{s}.{off}")
                ds.save_as(os.path.join(root, f"P{p}", name, f"IM{s:03d}.dcm"))
            for m in mask_folders:
                mk = dicom.new_ct_slice((raw[k] > 1200).astype(np.int16), instance=inst, uid_suffix=f"m{p}.{s}")
                mk.save_as(os.path.join(root, f"P{p}", m, f"IM{s:03d}.dcm"))
    return raw, slope, inter


def test_roundtrip_explicit_and_implicit(tmp_path):
    px = (np.arange(48 * 40) % 4096 - 1024).astype(np.int16).reshape(48, 40)
    ds = dicom.new_ct_slice(px, 0.5, -1000.0, instance=7, slice_location=-12.5)
    ds.SeriesDescription = "test series"
    ds.save_as(str(tmp_path / "e.dcm"))
    r = dicom.dcmread(str(tmp_path / "e.dcm"))
    np.testing.assert_array_equal(r.pixel_array, px)
    assert (r.Rows, r.Columns, r.InstanceNumber) == (48, 40, 7)
    assert (float(r.RescaleSlope), float(r.RescaleIntercept), float(r.SliceLocation)) == (0.5, -1000.0, -12.5)
    assert r.SeriesDescription == "test series" and r.get("PatientID", "none") == "none"
    # implicit VR little endian keeps every value
    r.file_meta.TransferSyntaxUID = dicom.IMPLICIT_VR_LE
    r.save_as(str(tmp_path / "i.dcm"))
    r2 = dicom.dcmread(str(tmp_path / "i.dcm"))
    np.testing.assert_array_equal(r2.pixel_array, px)
    assert r2.InstanceNumber == 7 and float(r2.RescaleSlope) == 0.5
    # stop_before_pixels
    assert "PixelData" not in dicom.dcmread(str(tmp_path / "e.dcm"), stop_before_pixels=True)


def test_undefined_length_sequence_is_carried_through(tmp_path):
    px = np.zeros((4, 4), np.int16)
    ds = dicom.new_ct_slice(px)
    # (0008,1140) SQ, undefined length, one undefined-length item holding a UI element
    item = struct.pack("<HH", 0x0008, 0x1155) + b"UI" + struct.pack("<H", 4) + b"1.2\x00"
    seq = (struct.pack("<HHI", 0xFFFE, 0xE000, 0xFFFFFFFF) + item + struct.pack("<HHI", 0xFFFE, 0xE00D, 0)
           + struct.pack("<HHI", 0xFFFE, 0xE0DD, 0))
    ds._el[0x00081140] = dicom.Element(0x00081140, "SQ", seq, undefined=True)
    ds.save_as(str(tmp_path / "s.dcm"))
    r = dicom.dcmread(str(tmp_path / "s.dcm"))
    assert r._el[0x00081140].raw == seq and r.Rows == 4
    c = copy.deepcopy(r)
    c.PixelData = np.ones((4, 4), np.int16).tobytes()
    assert r.pixel_array.sum() == 0 and c.pixel_array.sum() == 16


def test_dataset_pairs_and_orders_slices(tmp_path):
    raw, slope, inter = _write_tree(str(tmp_path))
    args = type("A", (), dict(ncct_folder="POST VUE", cect_folder="POST STD", use_masks=True,
                              auto_generate_masks=True, mask_types=["bone", "mediastinum"], mask_folders=[]))()
    dirs = sorted(str(tmp_path / p) for p in ("P0", "P1"))
    ds = DicomDataset(dirs, args)
    assert len(ds) == 6
    # InstanceNumber order: slice files IM002, IM001, IM000 (instances 1, 2, 3)
    it = ds[0]
    np.testing.assert_array_equal(it["A_raw"].numpy(), raw[2])
    np.testing.assert_array_equal(it["B_raw"].numpy(), raw[2] + 7)
    assert it["A_rescale"].tolist() == [float(slope[2]), float(inter[2])]
    b = collate([ds[i] for i in range(4)])
    assert b["A_raw"].shape == (4, 32, 32) and b["A_rescale"].shape == (4, 2)


def test_dataset_mask_files(tmp_path):
    raw, _, _ = _write_tree(str(tmp_path), patients=1, mask_folders=("bone_mask",))
    args = type("A", (), dict(ncct_folder="POST VUE", cect_folder="POST STD", use_masks=True,
                              auto_generate_masks=False, mask_types=[], mask_folders=["bone_mask", "mediastinum_mask"]))()
    ds = DicomDataset([str(tmp_path / "P0")], args)
    it = ds[0]
    assert it["mask_files"].shape == (2, 32, 32)
    np.testing.assert_array_equal(it["mask_files"][0].numpy(), (raw[2] > 1200).astype(np.float32))
    assert torch.isnan(it["mask_files"][1]).all()   # missing folder -> zero plane after preprocessing


def test_mixed_sizes_collate_to_list():
    a = {"A_raw": torch.zeros(4, 4, dtype=torch.int16), "A_rescale": torch.zeros(2)}
    b = {"A_raw": torch.zeros(6, 6, dtype=torch.int16), "A_rescale": torch.zeros(2)}
    out = collate([a, b])
    assert isinstance(out, list) and out[1]["A_raw"].shape == (1, 6, 6)


def test_preprocessing_needs_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from modules import mask_generator
    with pytest.raises(RuntimeError):
        mask_generator.detect_lung(np.zeros((8, 8), np.float32))
