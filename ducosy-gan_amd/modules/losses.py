"""Loss modules of the G step on the HIP kernels (modules/trainer.py:22-184, 347-351).

Same class names and constructor signatures as the reference; each forward is one fused
kernel sequence that produces the value AND d(value)/d(pred); the autograd backward only
rescales the saved gradient by the incoming scalar on the device (no host sync).
``SSIM`` is the drop-in for ``pytorch_msssim.SSIM(data_range, size_average=True, channel=1)``.
"""
import torch
import torch.nn as nn

from . import parallel
from .hip import ops

# the batch-coupled losses (ContrastRegion mean/std, ContrastEdge mean/std/top-10 %).
# The reference's nn.DataParallel (trainer.py:333-338) evaluates them on the whole batch gathered
# on cuda:0, so with more than one replica they are computed over the whole data-parallel batch
# by default (option ii, a few small all-reduces per evaluation).  GLOBAL_STATS = False
# (train.py --per_rank_loss_stats) uses each rank's shard instead (option i: DDP semantics).
# None = the default (whole batch); a module's own ``global_stats`` argument overrides it.
GLOBAL_STATS = None


def _global(flag):
    mode = GLOBAL_STATS if flag is None else flag
    return (True if mode is None else bool(mode)) and parallel.world() > 1


def stats_mode() -> str:
    """Which statistics the batch-coupled losses use in this process (printed at start-up)."""
    if parallel.world() == 1:
        return "single replica (whole batch)"
    return "whole data-parallel batch" if _global(None) else "per rank (--per_rank_loss_stats)"


class _FusedLoss(torch.autograd.Function):
    """value = fn(pred, *rest); backward: d/dpred = saved_grad * grad_out."""

    @staticmethod
    def forward(ctx, fn, pred, *rest):
        v, g = fn(pred, *rest, want_grad=ctx.needs_input_grad[1])
        ctx.g = g
        ctx.nrest = len(rest)
        return v

    @staticmethod
    def backward(ctx, gout):
        g = ops.scale_dev(ctx.g, gout.contiguous()) if ctx.g is not None else None
        ctx.g = None
        return (None, g) + (None,) * ctx.nrest


def _apply(fn, pred, *rest):
    return _FusedLoss.apply(fn, pred, *rest)


class L1Loss(nn.Module):
    """nn.L1Loss() (mean) — trainer.py:348-349."""

    def forward(self, pred, target):
        return _apply(lambda p, t, want_grad: ops.loss_l1(p, t, want_grad), pred, target)


class MSELoss(nn.Module):
    """nn.MSELoss() (mean) — trainer.py:347.  A python float target (the all-ones/all-zeros
    label maps of trainer.py:459-460) skips materialising the label tensor."""

    def forward(self, pred, target):
        if isinstance(target, (int, float)):
            return _apply(lambda p, want_grad: ops.loss_mse_const(p, float(target), want_grad), pred)
        return _apply(lambda p, t, want_grad: ops.loss_mse(p, t, want_grad), pred, target)


class GradientLoss(nn.Module):
    """trainer.py:22-40."""

    def forward(self, pred, target):
        return _apply(lambda p, t, want_grad: ops.loss_gradient(p, t, want_grad), pred, target)


class ContrastAttentionLoss(nn.Module):
    """trainer.py:43-86."""

    def __init__(self, sigma=0.1, min_weight=1.0, max_weight=3.0, blur_kernel=5):
        super().__init__()
        self.sigma, self.min_weight, self.max_weight = sigma, min_weight, max_weight
        self.blur_kernel = blur_kernel
        self.blur = nn.AvgPool2d(kernel_size=blur_kernel, stride=1, padding=blur_kernel // 2)

    def forward(self, pred, target, source):
        return _apply(lambda p, t, s, want_grad: ops.loss_contrast_attention(
            p, t, s, self.sigma, self.min_weight, self.max_weight, self.blur_kernel, want_grad),
            pred, target, source)


class ContrastRegionLoss(nn.Module):
    """trainer.py:89-130 (statistics over the whole batch tensor, unbiased std)."""

    def __init__(self, threshold=0.3, weight=2.0, global_stats=None):
        super().__init__()
        self.threshold, self.weight = threshold, weight
        self.global_stats = global_stats  # None: module default GLOBAL_STATS
        self.pool = nn.AvgPool2d(kernel_size=8, stride=8)

    def forward(self, pred, target, source):
        if _global(self.global_stats):
            return _apply(lambda p, t, s, want_grad: ops.loss_contrast_region_global(
                p, t, s, self.threshold, self.weight, parallel.allreduce_sum_, parallel.world(), want_grad),
                pred, target, source)
        return _apply(lambda p, t, s, want_grad: ops.loss_contrast_region(
            p, t, s, self.threshold, self.weight, want_grad), pred, target, source)


class ContrastEdgeLoss(nn.Module):
    """trainer.py:133-184 (exact top-10 % by radix select)."""

    def __init__(self, global_stats=None):
        super().__init__()
        self.global_stats = global_stats
        self.register_buffer("sobel_x", torch.tensor([[-1, 0, 1], [-2, 0, 2], [-1, 0, 1]],
                                                     dtype=torch.float32).view(1, 1, 3, 3))
        self.register_buffer("sobel_y", torch.tensor([[-1, -2, -1], [0, 0, 0], [1, 2, 1]],
                                                     dtype=torch.float32).view(1, 1, 3, 3))

    def forward(self, pred, target, source=None):
        if _global(self.global_stats):
            return _apply(lambda p, t, want_grad: ops.loss_contrast_edge_global(
                p, t, parallel.allreduce_sum_, parallel.world(), want_grad), pred, target)
        return _apply(lambda p, t, want_grad: ops.loss_contrast_edge(p, t, want_grad), pred, target)


class SSIM(nn.Module):
    """Drop-in for pytorch_msssim.SSIM (size_average=True, single-channel planes)."""

    def __init__(self, data_range=255, size_average=True, win_size=11, win_sigma=1.5, channel=3,
                 spatial_dims=2, K=(0.01, 0.03), nonnegative_ssim=False):
        super().__init__()
        if not size_average or nonnegative_ssim or spatial_dims != 2:
            raise NotImplementedError("SSIM: only size_average=True, 2-d, signed SSIM is on the hot path")
        self.data_range, self.win_size, self.win_sigma, self.K = data_range, win_size, win_sigma, K

    def forward(self, X, Y):
        if X.shape != Y.shape:
            raise ValueError(f"Input images should have the same dimensions, but got {X.shape} and {Y.shape}.")
        return _apply(lambda x, y, want_grad: ops.loss_ssim(x, y, self.data_range, self.win_size,
                                                            self.win_sigma, self.K, want_grad), X, Y)
