"""Argument sets of the reference's modules/argmanager.py (same flags, defaults and fixed
per-target Namespaces) plus the flags this build adds for the MI355X trainer.

Reference: modules/argmanager.py:4-44 (inference), :84-119 (common training args),
:122-152 (soft-tissue / lung fixed args).  ``argv`` may be passed explicitly (the reference
always parses sys.argv; with ``argv=None`` so does this module).
"""
from __future__ import annotations

import argparse
import os


def _add_build_train_flags(p: argparse.ArgumentParser):
    """Flags that exist only in this build (all default to the reference's behaviour)."""
    g = p.add_argument_group("MI355X build")
    g.add_argument("--synthetic", action="store_true",
                   help="train on deterministic synthetic slices (U(-1,1) images, Bernoulli(0.3) masks) "
                        "instead of the DICOM dataset")
    g.add_argument("--synthetic_slices", type=int, default=64, help="number of synthetic training slices")
    g.add_argument("--num_residual_blocks", type=int, default=9, help="Generator residual blocks (reference: 9)")
    g.add_argument("--max_steps_per_epoch", type=int, default=0, help="cap on steps per epoch (0 = full epoch)")
    g.add_argument("--log_every", type=int, default=10, help="print losses every N steps (rank 0)")
    g.add_argument("--seed", type=int, default=0, help="torch seed for weight initialisation")
    g.add_argument("--global_loss_stats", action="store_true",
                   help="at N GPUs, compute the batch-coupled losses (ContrastRegion, ContrastEdge) over the "
                        "whole data-parallel batch, the reference's semantics (the default; kept for scripts)")
    g.add_argument("--per_rank_loss_stats", action="store_true",
                   help="at N GPUs, compute the batch-coupled losses on each rank's shard (DDP semantics; no "
                        "collectives inside the losses) instead of over the whole batch")


def get_common_infer_args(argv=None):
    """modules/argmanager.py:4-44."""
    p = argparse.ArgumentParser(description="CycleGAN Inference for CT Scans")
    p.add_argument("--data_dir_root", type=str, default="./data")
    p.add_argument("--input_dir_root", type=str, default="/archive/Dataset_DuCoSyGAN")
    p.add_argument("--working_dir_root", type=str, default="./data/working")
    p.add_argument("--output_dir_root", type=str, default="./data/output")
    p.add_argument("--dataset_names", type=str, nargs="+", default=["Kangwon_National_Univ_Masked_10"])
    p.add_argument("--ncct_folder", type=str, default="POST VUE")
    p.add_argument("--cect_folder", type=str, default="POST STD")
    p.add_argument("--apply_masking", action="store_true")
    p.add_argument("--img_size", type=int, default=512)
    p.add_argument("--batch_size", type=int, default=4)
    p.add_argument("--nmodel_path", type=str, default="./checkpoints/Normal_Map_Unet.pth")
    p.add_argument("--window_center", type=int, default=40)
    p.add_argument("--window_width", type=int, default=400)
    p.add_argument("--gpu_id", type=int, default=0)
    p.add_argument("--fast", action="store_true")
    p.add_argument("--reset", action="store_true")
    p.add_argument("--mask", action="store_true")
    p.add_argument("--skip_convert", action="store_true")
    args, _ = p.parse_known_args(argv)
    for d in (args.data_dir_root, args.working_dir_root, args.output_dir_root):
        os.makedirs(d, exist_ok=True)
    return args


def get_soft_tissue_infer_args(argv=None):
    """modules/argmanager.py:47-63."""
    p = argparse.ArgumentParser(description="CycleGAN Inference for CT Scans")
    p.add_argument("--model_path", type=str, default="./checkpoints/v3/Soft_Tissue_Generator_A2B.pth")
    p.add_argument("--hu_min", type=int, default=-150)
    p.add_argument("--hu_max", type=int, default=250)
    args, _ = p.parse_known_args(argv)
    return args


def get_lung_infer_args(argv=None):
    """modules/argmanager.py:66-81."""
    p = argparse.ArgumentParser(description="CycleGAN Inference for CT Scans")
    p.add_argument("--model_path", type=str, default="./checkpoints/v3/Lung_Generator_A2B.pth")
    p.add_argument("--hu_min", type=int, default=-1000)
    p.add_argument("--hu_max", type=int, default=-150)
    args, _ = p.parse_known_args(argv)
    return args


def get_common_train_args(argv=None):
    """modules/argmanager.py:84-119.  ``--batch_size`` is the TOTAL batch across GPUs, as in
    the reference (:95); each of the W processes trains on batch_size // W slices."""
    p = argparse.ArgumentParser(description="Common Training Arguments for CycleGAN")
    p.add_argument("--target_model", type=str, default="soft_tissue", choices=["soft_tissue", "lung", "all"])
    p.add_argument("--epochs", type=int, default=10000)
    p.add_argument("--decay_epoch", type=int, default=100)
    p.add_argument("--batch_size", type=int, default=8, help="Total batch size across all GPUs")
    p.add_argument("--lr", type=float, default=0.0002)
    p.add_argument("--lambda_cyc", type=float, default=10.0)
    p.add_argument("--lambda_id", type=float, default=5.0)
    p.add_argument("--num_workers", type=int, default=16)
    p.add_argument("--training_dir", type=str, default="./training_dir")
    p.add_argument("--data_root", type=str, default="/workspace/Contrast_CT/hyunsu/Dataset_DucosyGAN")
    p.add_argument("--dataset_names", type=str, default="Kangwon_National_Univ_Masked_10")
    p.add_argument("--ncct_folder", type=str, default="POST VUE")
    p.add_argument("--cect_folder", type=str, default="POST STD")
    p.add_argument("--resume", type=str, default="checkpoint.pth.tar")
    p.add_argument("--img_size", type=int, default=512)
    p.add_argument("--val_split", type=float, default=0.2)
    _add_build_train_flags(p)
    args = p.parse_args(argv)
    os.makedirs(args.training_dir, exist_ok=True)
    return args


def get_soft_tissue_train_args():
    """modules/argmanager.py:122-137 (fixed values)."""
    return argparse.Namespace(hu_min=-150, hu_max=250, window_width=400, window_center=40,
                              use_soft_squeezing=True, use_cbam=True, use_masks=True, auto_generate_masks=True,
                              mask_types=["bone", "mediastinum"], mask_folders=["bone_mask", "mediastinum_mask"])


def get_lung_train_args():
    """modules/argmanager.py:140-152 (fixed values)."""
    return argparse.Namespace(hu_min=-1000, hu_max=-150, window_width=1500, window_center=-600,
                              use_soft_squeezing=True, use_cbam=True, use_masks=True, auto_generate_masks=True,
                              mask_types=["lung"], mask_folders=["lung_mask"])
