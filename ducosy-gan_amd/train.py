"""Training entry point — mirror of the reference's train.py:1-46.

    python ducosy-gan_amd/train.py --target_model soft_tissue --synthetic --epochs 2
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        ducosy-gan_amd/train.py --batch_size 64 ...

One process per GPU (torchrun env); ``--batch_size`` is the global batch as in the reference.
"""
import os
import sys
import warnings
from argparse import Namespace

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from modules.argmanager import get_common_train_args, get_lung_train_args, get_soft_tissue_train_args  # noqa: E402
from modules.trainer import train_cycle_gan  # noqa: E402

warnings.filterwarnings("ignore", category=UserWarning, module="pydicom")


def combine_args(common_args, train_args):
    """train.py:8-14: common flags overlaid with the target's fixed arguments."""
    args = vars(common_args).copy()
    args.update(vars(train_args))
    return Namespace(**args)


def train(train_args):
    """train.py:16-38."""
    target_model = train_args.target_model.lower()
    if target_model not in ["soft_tissue", "lung", "all"]:
        raise ValueError("Invalid target_model. Choose from 'soft_tissue', 'lung', or 'all'.")
    if target_model in ("soft_tissue", "all"):
        print("Starting training for Soft-tissue CycleGAN...")
        train_cycle_gan(combine_args(train_args, get_soft_tissue_train_args()), target_range="soft_tissue")
        print("Soft-tissue CycleGAN training completed.")
    if target_model in ("lung", "all"):
        print("Starting training for Lung CycleGAN...")
        train_cycle_gan(combine_args(train_args, get_lung_train_args()), target_range="lung")
        print("Lung CycleGAN training completed.")


if __name__ == "__main__":
    print("Starting DUCOSY-GAN Training Process")
    train(get_common_train_args())
    print("DUCOSY-GAN Training Process Completed")
