"""GPU path of the input pipeline drop-ins: modules/dataset.py's SliceBatchPreprocessor (decoded
DICOM batch -> the reference's {"A", "B", "masks"} batch), the modules/mask_generator.py and
modules/preprocess.py functions with the reference's signatures, and one train_cycle_gan epoch
reading a DICOM tree end to end.  Checked against the oracle (oracle/masks_ref.py, itself
pinned to the reference by tests/golden/masks_*.npz)."""
import argparse
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from modules import dicom, mask_generator, phantom, preprocess
from modules.dataset import DicomDataset, SliceBatchPreprocessor, collate
from oracle import masks_ref
from test_cpu_dicom import _write_tree

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _args(**kw):
    a = dict(ncct_folder="POST VUE", cect_folder="POST STD", use_masks=True, auto_generate_masks=True,
             mask_types=["bone", "mediastinum"], mask_folders=["bone_mask", "mediastinum_mask"], hu_min=-150,
             hu_max=250, use_soft_squeezing=True, img_size=128)
    a.update(kw)
    return argparse.Namespace(**a)


def _oracle_batch(raw, slope, inter, args, idx, kw):
    A, M = [], []
    for k in idx:
        hu, img = masks_ref.hu_transform(raw[k], slope[k], inter[k], args.hu_min, args.hu_max, args.use_soft_squeezing)
        A.append(img)
        M.append(masks_ref.masks_batch(hu[None], args.mask_types, **kw)[0])
    return np.stack(A)[:, None], np.stack(M)


def test_preprocessor_matches_oracle(tmp_path):
    raw, slope, inter = _write_tree(str(tmp_path), patients=1, slices=4, size=128)
    args = _args()
    ds = DicomDataset([str(tmp_path / "P0")], args)
    batch = collate([ds[i] for i in range(4)])
    kw = dict(min_size=64, border_margin=32)
    # the dataset path uses the reference defaults; at 128x128 the border margin of 32 still
    # leaves a 64x64 interior, enough for the phantom's lungs
    out = SliceBatchPreprocessor(args, DEV)(batch)
    order = [3, 2, 1, 0]  # InstanceNumber order of the written tree
    want_a, want_m = _oracle_batch(raw, slope, inter, args, order, kw)
    np.testing.assert_allclose(out["A"].cpu().numpy(), want_a, rtol=0, atol=2e-7)
    np.testing.assert_array_equal(out["masks"].cpu().numpy(), want_m)
    assert out["B"].shape == (4, 1, 128, 128)


def test_preprocessor_resizes_like_the_transform(tmp_path):
    raw, slope, inter = _write_tree(str(tmp_path), patients=1, slices=2, size=96)
    args = _args(img_size=64, mask_types=["lung", "bone"])
    ds = DicomDataset([str(tmp_path / "P0")], args)
    out = SliceBatchPreprocessor(args, DEV)(collate([ds[0], ds[1]]))
    want_a, want_m = _oracle_batch(raw, slope, inter, args, [1, 0], dict(min_size=64, border_margin=32))
    ra = F.interpolate(torch.from_numpy(want_a), size=(64, 64), mode="bilinear", align_corners=False, antialias=True)
    rm = F.interpolate(torch.from_numpy(want_m), size=(64, 64), mode="nearest")
    np.testing.assert_allclose(out["A"].cpu().numpy(), ra.numpy(), rtol=0, atol=1e-6)
    np.testing.assert_array_equal(out["masks"].cpu().numpy(), rm.numpy())


def test_mask_generator_dropin_2d_3d():
    hu = np.stack([phantom.slice_hu(61, i, 160) for i in range(5)]).astype(np.float32)
    kw = dict(min_size=64, border_margin=32)
    want = masks_ref.masks_batch(hu, ("lung", "mediastinum", "bone", "lung_vessel"), **kw)
    lung3 = mask_generator.detect_lung(hu)                                   # 3-D volume
    assert lung3.dtype == np.uint8 and lung3.shape == hu.shape
    np.testing.assert_array_equal(lung3, want[:, 0])
    np.testing.assert_array_equal(mask_generator.detect_mediastinum(hu, lung3), want[:, 1])
    np.testing.assert_array_equal(mask_generator.detect_bone(hu, lung3), want[:, 2])
    np.testing.assert_array_equal(mask_generator.detect_lung_vessels(hu, lung3), want[:, 3])
    m2 = mask_generator.generate_anatomical_masks(hu[0], ["bone", "lung"])  # 2-D slice
    assert set(m2) == {"bone", "lung"}
    np.testing.assert_array_equal(m2["bone"], want[0, 2])
    # a lung mask from elsewhere (here: eroded) drives the hull, as the reference's argument does
    lung_other = lung3.copy()
    lung_other[:, :, :80] = 0
    got = mask_generator.detect_mediastinum(torch.from_numpy(hu).to(DEV), torch.from_numpy(lung_other).to(DEV))
    for z in range(hu.shape[0]):
        body = hu[z] > -1000
        gate = masks_ref._lung_gate(lung_other[z], body)
        if gate:
            inside, ok = masks_ref._hull_inside(lung_other[z])
            exp = (inside != lung_other[z].astype(bool)) & (hu[z] >= -300) & (hu[z] <= 450)
        else:
            exp = np.zeros_like(body)
        np.testing.assert_array_equal(got[z].cpu().numpy(), exp.astype(np.uint8))


def test_preprocess_dropins(tmp_path):
    raw, slope, inter = phantom.ct_batch(71, 2, 64)
    ds = dicom.new_ct_slice(raw[0], float(slope[0]), float(inter[0]))
    ds.save_as(str(tmp_path / "x.dcm"))
    d = dicom.dcmread(str(tmp_path / "x.dcm"))
    _, want = masks_ref.hu_transform(raw[0], slope[0], inter[0], -1000, -150, True)
    np.testing.assert_allclose(preprocess.apply_hu_transform(d, -1000, -150), want, rtol=0, atol=2e-7)
    _, lin = masks_ref.hu_transform(raw[0], slope[0], inter[0], -150, 250, False)
    np.testing.assert_array_equal(preprocess.apply_hu_transform(d, -150, 250, False), lin)
    soft_t, lung_t, _ = preprocess.preprocess_dicom(str(tmp_path / "x.dcm"), -150, 250, -1000, -150)
    np.testing.assert_array_equal(soft_t[0].numpy(), lin)
    back = preprocess.postprocess_tensor(soft_t, d, -150, 250)
    assert back.dtype == np.int16


def test_train_epoch_on_a_dicom_tree(tmp_path):
    """train_cycle_gan reading DICOM: decode on the loader, HU transform + masks on the GPU."""
    from modules.trainer import train_cycle_gan
    data = tmp_path / "data" / "DS"
    _write_tree(str(data), patients=3, slices=2, size=64)
    a = _args(img_size=64)
    a.__dict__.update(dict(data_root=str(tmp_path / "data"), dataset_names="DS", training_dir=str(tmp_path / "td"),
                           batch_size=2, epochs=1, decay_epoch=0, lr=2e-4, lambda_cyc=10.0, lambda_id=5.0,
                           num_workers=0, val_split=0.34, resume="", window_center=40, window_width=400,
                           num_residual_blocks=1, max_steps_per_epoch=2, log_every=1, seed=0, synthetic=False))
    system = train_cycle_gan(a, "soft_tissue")
    assert system.G_A2B.input_channels == 3
    saved = os.listdir(tmp_path / "td" / "soft_tissue" / "saved_models")
    assert "checkpoint.pth.tar" in saved and "G_A2B_last.pth" in saved


def test_generate_and_synthesis_end_to_end(tmp_path):
    """generate.py on a DICOM tree with mask-conditioned checkpoints (soft cin 3, lung cin 2):
    raw / soft_tissue / lung copies, then the merged, z-smoothed output series."""
    import importlib.util
    from conftest import ROOT
    from modules.model import Generator
    spec = importlib.util.spec_from_file_location("dcs_gen", os.path.join(ROOT, "ducosy-gan_amd", "generate.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    _write_tree(str(tmp_path / "in" / "DS"), patients=1, slices=3, size=64)
    torch.manual_seed(0)
    paths = {}
    for name, cin in (("soft", 3), ("lung", 2)):
        paths[name] = str(tmp_path / f"{name}.pth")
        torch.save(Generator(cin, 9).state_dict(), paths[name])
    a = gen.get_args(["--input_dir_root", str(tmp_path / "in"), "--working_dir_root", str(tmp_path / "w"),
                      "--output_dir_root", str(tmp_path / "o"), "--dataset_names", "DS", "--img_size", "64",
                      "--model_path_soft", paths["soft"], "--model_path_lung", paths["lung"]])
    gen.generate(a)
    gen.synthesis(a)
    for k in ("raw", "soft_tissue", "lung"):
        assert len(os.listdir(tmp_path / "w" / "DS" / "P0" / k)) == 3
    outs = sorted(os.listdir(tmp_path / "o" / "DS" / "P0"))
    assert outs == ["0000.dcm", "0001.dcm", "0002.dcm"]
    o = dicom.dcmread(str(tmp_path / "o" / "DS" / "P0" / "0000.dcm"))
    assert o.pixel_array.shape == (64, 64) and o.SeriesDescription == "DuCoSyGAN sCECT v2"


def test_generate_reference_signature(tmp_path):
    """generate(args, soft_tissue_args, lung_args) / synthesis(...) as the reference calls them
    (generate.py:21, 137; modules/argmanager.py:4-82 namespaces) give the same files as the
    single-parser form."""
    import argparse
    import importlib.util
    from conftest import ROOT
    from modules.model import Generator
    spec = importlib.util.spec_from_file_location("dcs_gen2", os.path.join(ROOT, "ducosy-gan_amd", "generate.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    _write_tree(str(tmp_path / "in" / "DS"), patients=1, slices=2, size=64)
    torch.manual_seed(1)
    paths = {}
    for name, cin in (("soft", 3), ("lung", 2)):
        paths[name] = str(tmp_path / f"{name}.pth")
        torch.save(Generator(cin, 9).state_dict(), paths[name])
    outs = []
    for form in ("single", "reference"):
        w, o = tmp_path / f"w_{form}", tmp_path / f"o_{form}"
        a = gen.get_args(["--input_dir_root", str(tmp_path / "in"), "--working_dir_root", str(w),
                          "--output_dir_root", str(o), "--dataset_names", "DS", "--img_size", "64",
                          "--model_path_soft", paths["soft"], "--model_path_lung", paths["lung"]])
        if form == "single":
            gen.generate(a)
            gen.synthesis(a)
        else:
            soft = argparse.Namespace(model_path=paths["soft"], hu_min=-150, hu_max=250)
            lung = argparse.Namespace(model_path=paths["lung"], hu_min=-1000, hu_max=-150)
            gen.generate(a, soft, lung)
            gen.synthesis(a, soft, lung)
        outs.append([dicom.dcmread(str(o / "DS" / "P0" / f)).pixel_array for f in ("0000.dcm", "0001.dcm")])
    for x, y in zip(*outs):
        assert np.array_equal(x, y)
