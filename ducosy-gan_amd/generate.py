"""Inference entry point — mirror of the reference's generate.py (generate(), synthesis()).

    python ducosy-gan_amd/generate.py --input_dir_root ... --dataset_names NAME \
        --model_path_soft ckpt_soft.pth --model_path_lung ckpt_lung.pth

Differences from the reference, all deliberate:
  * slices of a patient are translated in batches on the MI355X Generator kernels
    (modules/inference.py) instead of one slice per call;
  * the Generators are built with the input channel count found in the checkpoint
    (generate.py:29-30 hard-codes 1, which cannot load the mask-conditioned cin 3 / cin 2
    checkpoints that train.py writes); a mask-conditioned Generator gets the anatomical masks
    of the NCCT slice in its training order (soft tissue: bone, mediastinum; lung: lung;
    modules/argmanager.py) from the GPU mask kernel, as the training data pipeline built them;
  * checkpoints are read with torch.load(weights_only=True).
DICOM reading/writing uses modules/dicom.py (pydicom is not installed in this image).
"""
import argparse
import glob
import os
import shutil
import sys
import traceback
from copy import deepcopy

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from modules.inference import (hu_from_stored, normalise_hu, smooth_volume, stored_from_output,  # noqa: E402
                               synthesize, translate_slices)
from modules.model import Generator  # noqa: E402


def load_generator(path, device, num_residual_blocks=9):
    """Generator with the checkpoint's own input channel count (module.-prefix tolerant)."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if all(k.startswith("module.") for k in sd):
        sd = {k[len("module."):]: v for k, v in sd.items()}
    cin = int(sd["model.1.weight"].shape[1])
    g = Generator(input_channels=cin, num_residual_blocks=num_residual_blocks)
    g.load_state_dict(sd)
    return g.to(device).eval()


MASK_TYPES = {"soft_tissue": ["bone", "mediastinum"], "lung": ["lung"]}  # argmanager.py:132, 149


def _conditioning(g, kind, hu_slices, device):
    """Per-slice mask channels for a mask-conditioned Generator (None for an image-only one):
    the training mask types when their count matches the checkpoint, else zero planes."""
    extra = g.input_channels - 1
    if extra <= 0:
        return None
    types = MASK_TYPES[kind]
    if len(types) != extra:
        return [np.zeros((extra,) + h.shape, np.float32) for h in hu_slices]
    from modules.hip import ops
    out = []
    for h in hu_slices:
        m = ops.anatomical_masks(torch.from_numpy(np.ascontiguousarray(h, np.float32)).to(device), types)
        out.append(m[0].cpu().numpy())
    return out


def _model_args(args, soft_tissue_args, lung_args):
    """The reference passes the per-model settings as two extra namespaces (model_path, hu_min,
    hu_max; modules/argmanager.py:52-82); this build's single parser carries them as
    --model_path_soft / --soft_hu_min / ... on ``args``.  Either form is accepted."""
    if soft_tissue_args is None:
        soft_tissue_args = argparse.Namespace(model_path=args.model_path_soft, hu_min=args.soft_hu_min,
                                              hu_max=args.soft_hu_max)
    if lung_args is None:
        lung_args = argparse.Namespace(model_path=args.model_path_lung, hu_min=args.lung_hu_min,
                                       hu_max=args.lung_hu_max)
    return soft_tissue_args, lung_args


def generate(args, soft_tissue_args=None, lung_args=None):
    """generate.py:21-137 (same signature): per patient, translate every NCCT slice with both
    models and write raw / soft_tissue / lung DICOM copies under working_dir_root."""
    from modules import dicom
    sa, la = _model_args(args, soft_tissue_args, lung_args)
    device = torch.device(f"cuda:{args.gpu_id}")
    soft = load_generator(sa.model_path, device)
    lung = load_generator(la.model_path, device)
    batch = int(getattr(args, "slice_batch", 16))
    for dataset_name in args.dataset_names:
        input_dir = os.path.join(args.input_dir_root, dataset_name)
        working_dir = os.path.join(args.working_dir_root, dataset_name)
        for patient_dir in sorted(d for d in glob.glob(os.path.join(input_dir, "*")) if os.path.isdir(d)):
            ncct = os.path.join(patient_dir, args.ncct_folder)
            if not os.path.isdir(ncct):
                continue
            out_dirs = {k: os.path.join(working_dir, os.path.basename(patient_dir), k)
                        for k in ("raw", "soft_tissue", "lung")}
            for d in out_dirs.values():
                os.makedirs(d, exist_ok=True)
            paths = sorted(glob.glob(os.path.join(ncct, "*.dcm")))
            dcms = [dicom.dcmread(p) for p in paths]
            hu = [hu_from_stored(d.pixel_array, d.RescaleSlope, d.RescaleIntercept) for d in dcms]
            outs = {}
            for name, model, lo, hi in (("soft_tissue", soft, sa.hu_min, sa.hu_max),
                                        ("lung", lung, la.hu_min, la.hu_max)):
                outs[name] = (translate_slices(model, [normalise_hu(h, lo, hi) for h in hu], args.img_size,
                                               batch, device, _conditioning(model, name, hu, device)),
                              lo, hi)
            for i, (p, d) in enumerate(zip(paths, dcms)):
                try:
                    shutil.copy(p, os.path.join(out_dirs["raw"], os.path.basename(p)))
                    for name, (ys, lo, hi) in outs.items():
                        px = stored_from_output(ys[i], lo, hi, d.RescaleSlope, d.RescaleIntercept,
                                                d.pixel_array.dtype)
                        o = deepcopy(d)
                        o.SeriesDescription = f"Synthetic CECT (from {d.get('SeriesDescription', '')})"
                        o.file_meta.TransferSyntaxUID = dicom.EXPLICIT_VR_LE
                        o.SmallestImagePixelValue, o.LargestImagePixelValue = int(px.min()), int(px.max())
                        o.PixelData = px.tobytes()
                        o.save_as(os.path.join(out_dirs[name], os.path.basename(p)))
                except Exception as e:  # the reference reports and continues (generate.py:131-135)
                    print(f"Could not process file {p}. Error: {e}")
                    traceback.print_exc()
    print("\nGeneration complete.")


def synthesis(args, soft_tissue_args=None, lung_args=None):
    """generate.py:137-297 (same signature): merge the two translations inside their HU ranges
    over the NCCT, z-smooth the volume (modules/postprocess.py) and write
    output/{dataset}/{patient}/{idx:04d}.dcm."""
    from modules import dicom
    sa, la = _model_args(args, soft_tissue_args, lung_args)
    for dataset_name in args.dataset_names:
        working_dir = os.path.join(args.working_dir_root, dataset_name)
        output_dir = os.path.join(args.output_dir_root, dataset_name)
        for patient_dir in sorted(d for d in glob.glob(os.path.join(working_dir, "*")) if os.path.isdir(d)):
            lists = [sorted(glob.glob(os.path.join(patient_dir, k, "*.dcm"))) for k in ("raw", "soft_tissue", "lung")]
            if not all(lists) or len({len(x) for x in lists}) != 1:
                print(f"Skipping {patient_dir}: missing or mismatched slices")
                continue
            merged = []
            for rp, sp, lp in zip(*lists):
                raw, st, lg = dicom.dcmread(rp), dicom.dcmread(sp), dicom.dcmread(lp)
                raw_hu = hu_from_stored(raw.pixel_array, getattr(raw, "RescaleSlope", 1),
                                        getattr(raw, "RescaleIntercept", 0))
                merged.append(synthesize(raw.pixel_array, raw_hu, st.pixel_array, lg.pixel_array,
                                         (sa.hu_min, sa.hu_max), (la.hu_min, la.hu_max)))
            vol = smooth_volume(merged)
            out_base = os.path.join(output_dir, os.path.basename(patient_dir))
            os.makedirs(out_base, exist_ok=True)
            for idx, sp in enumerate(lists[1]):
                o = dicom.dcmread(sp)
                px = vol[idx]
                o.PixelData = px.tobytes()
                vr = "US" if o.PixelRepresentation == 0 else "SS"
                o.add_new((0x0028, 0x0106), vr, int(px.min()))
                o.add_new((0x0028, 0x0107), vr, int(px.max()))
                o.WindowWidth, o.WindowCenter = 1250, -375.0   # generate.py:279-282
                o.SeriesDescription = "DuCoSyGAN sCECT v2"
                o.save_as(os.path.join(out_base, f"{idx:04d}.dcm"))
    print("\nSynthesis complete.")


def get_args(argv=None):
    """The reference's inference arguments (modules/argmanager.py:4-81) in one parser (the
    reference parses sys.argv three times with three parsers, generate.py:483-485)."""
    p = argparse.ArgumentParser(description="CycleGAN Inference for CT Scans (MI355X)")
    p.add_argument("--input_dir_root", default="/archive/Dataset_DuCoSyGAN")
    p.add_argument("--working_dir_root", default="./data/working")
    p.add_argument("--output_dir_root", default="./data/output")
    p.add_argument("--dataset_names", nargs="+", default=["Kangwon_National_Univ_Masked_10"])
    p.add_argument("--ncct_folder", default="POST VUE")
    p.add_argument("--img_size", type=int, default=512)
    p.add_argument("--gpu_id", type=int, default=0)
    p.add_argument("--slice_batch", type=int, default=16, help="slices per Generator call")
    p.add_argument("--model_path_soft", default="./checkpoints/v3/Soft_Tissue_Generator_A2B.pth")
    p.add_argument("--model_path_lung", default="./checkpoints/v3/Lung_Generator_A2B.pth")
    p.add_argument("--soft_hu_min", type=int, default=-150)
    p.add_argument("--soft_hu_max", type=int, default=250)
    p.add_argument("--lung_hu_min", type=int, default=-1000)
    p.add_argument("--lung_hu_max", type=int, default=-150)
    p.add_argument("--skip_convert", action="store_true", help="only run the synthesis stage")
    return p.parse_args(argv)


if __name__ == "__main__":
    a = get_args()
    soft_a, lung_a = _model_args(a, None, None)
    if not a.skip_convert:
        generate(a, soft_a, lung_a)
    synthesis(a, soft_a, lung_a)
