"""Drop-in mirror of the reference's modules/trainer.py on the MI355X kernel library.

* Loss classes with the reference's names/signatures (trainer.py:22-184) — fused HIP kernels
  (modules/losses.py).
* ``CycleGANSystem.train_step`` — the step loop body of trainer.py:447-531 (G step with nine
  loss terms, D_A step, D_B step, three Adam steps) on the fused Generator/Discriminator
  autograd Functions, with the reference's math but an MI355X-shaped schedule:
    - the two Generator calls that share weights and inputs of equal shape are batched
      (G_A2B on [real_A; real_B] gives fake_B and id_B at once; IN is per-sample, so results
      are identical), as are the two Discriminator calls of each D step;
    - the G-step Discriminator calls skip the parameter gradients the reference computes and
      then discards with optimizer_D.zero_grad() (trainer.py:470, :517);
    - each optimizer is one flat-buffer Adam launch; with >1 process one RCCL all-reduce per
      optimizer averages the flat gradient (modules/parallel.py).
* ``train_cycle_gan(args, target_range)`` — trainer.py:297-597: resume, per-epoch LambdaLR,
  validation, and the checkpoint layout (file names and checkpoint.pth.tar keys) unchanged.
"""
from __future__ import annotations

import glob
import math
import os
import random
import time

import torch
import torch.nn as nn

from . import parallel
from .losses import (L1Loss, MSELoss, SSIM, ContrastAttentionLoss, ContrastEdgeLoss,  # noqa: F401
                     ContrastRegionLoss, GradientLoss)
from .model import Discriminator, Generator, weights_init_normal
from .optim import FusedAdam

LAMBDA_GRAD, LAMBDA_GRAD_ID, LAMBDA_SSIM = 5.0, 2.5, 2.0        # trainer.py:493-495
LAMBDA_CA, LAMBDA_CR, LAMBDA_CE = 2.0, 1.5, 1.0                 # trainer.py:500-502

# The step as an explicit schedule of the fused forward / backward functions and the fused loss
# kernel (no autograd graph: no slice / cat backward fills and copies, no per-term scalar
# arithmetic, no gradient adds); False = the autograd step over the same kernels (the reference
# structure)
_EXPLICIT_STEP = True

# loss_G's output slots of the fused loss recipe (and the train_step dict keys)
_G_TERMS = ("loss_G", "loss_GAN", "loss_cycle", "loss_id", "loss_grad_cycle", "loss_grad_id", "loss_ssim",
            "loss_contrast_attention", "loss_contrast_region", "loss_contrast_edge")


def apply_windowing(tensor_img, args):
    """modules/preprocess.py:58-65 (used for the validation image grid)."""
    hu_img = (tensor_img + 1.0) / 2.0 * (args.hu_max - args.hu_min) + args.hu_min
    wc, ww = args.window_center, args.window_width
    lo, hi = wc - ww / 2.0, wc + ww / 2.0
    return (torch.clamp(hu_img, lo, hi) - lo) / ww


class CycleGANSystem:
    """G_A2B, G_B2A, D_A, D_B + criteria + three Adam optimizers (trainer.py:319-367)."""

    def __init__(self, input_channels=1, num_residual_blocks=9, use_cbam=True, lr=2e-4,
                 lambda_cyc=10.0, lambda_id=5.0, device="cuda", init=True):
        self.device = torch.device(device)
        mk = lambda: Generator(input_channels=input_channels, num_residual_blocks=num_residual_blocks,
                               use_cbam=use_cbam)
        self.G_A2B, self.G_B2A = mk(), mk()
        self.D_A, self.D_B = Discriminator(), Discriminator()
        if init:
            for m in (self.G_A2B, self.G_B2A, self.D_A, self.D_B):
                m.apply(weights_init_normal)
        for m in self.models:
            m.to(self.device)
        self.lambda_cyc, self.lambda_id = lambda_cyc, lambda_id
        self.criterion_GAN = MSELoss()
        self.criterion_cycle = L1Loss()
        self.criterion_identity = L1Loss()
        self.criterion_gradient = GradientLoss()
        self.criterion_ssim = SSIM(data_range=1.0, size_average=True, channel=1)
        self.criterion_contrast_attention = ContrastAttentionLoss(sigma=0.15, min_weight=1.0, max_weight=3.0,
                                                                  blur_kernel=7)
        self.criterion_contrast_region = ContrastRegionLoss(threshold=0.15, weight=1.5)
        self.criterion_contrast_edge = ContrastEdgeLoss().to(self.device)
        betas = (0.5, 0.999)
        self.optimizer_G = FusedAdam(list(self.G_A2B.parameters()) + list(self.G_B2A.parameters()), lr=lr,
                                     betas=betas)
        self.optimizer_D_A = FusedAdam(self.D_A.parameters(), lr=lr, betas=betas)
        self.optimizer_D_B = FusedAdam(self.D_B.parameters(), lr=lr, betas=betas)
        # identical initial replicas on every rank
        for opt in self.optimizers:
            parallel.broadcast_(opt.flat_p, 0)
        # the broadcast wrote every parameter through the flat buffer, behind the parameters' own
        # version counters: no packed weight built before it may be reused
        from .hip import ops
        ops.bump_weights_epoch()

    @property
    def models(self):
        return (self.G_A2B, self.G_B2A, self.D_A, self.D_B)

    @property
    def optimizers(self):
        return (self.optimizer_G, self.optimizer_D_A, self.optimizer_D_B)

    def train(self):
        for m in self.models:
            m.train()

    def train_step(self, real_A, real_B, masks=None):
        """One pass of trainer.py:463-525.  Returns the loss terms as 0-d device tensors (no
        host synchronisation inside)."""
        if _EXPLICIT_STEP:
            return self._train_step_explicit(real_A, real_B, masks)
        return self._train_step_autograd(real_A, real_B, masks)

    # ---- the step as an explicit schedule ---------------------------------------------------
    def _g_loss_recipe(self, njobs):
        """Coefficients composing _G_TERMS from the fused loss jobs' term means (job order of
        _train_step_explicit: 0 rec_A, 1 rec_B, 2 id_A, 3 id_B, 4 fake_B, 5 D_B(fake_B),
        6 D_A(fake_A); value q: 0 L1, 1/2 gradient x/y, 3 SSIM, 4 CA / MSE) and two extra scalars
        (ContrastRegion, ContrastEdge).  trainer.py:469-512."""
        lc, li = self.lambda_cyc, self.lambda_id
        terms = {
            "loss_GAN": ({(5, 4): .5, (6, 4): .5}, 0.0, (0, 0)),
            "loss_cycle": ({(0, 0): .5, (1, 0): .5}, 0.0, (0, 0)),
            "loss_id": ({(2, 0): .5, (3, 0): .5}, 0.0, (0, 0)),
            "loss_grad_cycle": ({(0, 1): .5, (0, 2): .5, (1, 1): .5, (1, 2): .5}, 0.0, (0, 0)),
            "loss_grad_id": ({(2, 1): .5, (2, 2): .5, (3, 1): .5, (3, 2): .5}, 0.0, (0, 0)),
            "loss_ssim": ({(0, 3): -.5, (1, 3): -.5}, 1.0, (0, 0)),
            "loss_contrast_attention": ({(4, 4): 1.0}, 0.0, (0, 0)),
            "loss_contrast_region": ({}, 0.0, (1, 0)),
            "loss_contrast_edge": ({}, 0.0, (0, 1)),
        }
        lam = {"loss_GAN": 1.0, "loss_cycle": lc, "loss_id": li, "loss_grad_cycle": LAMBDA_GRAD,
               "loss_grad_id": LAMBDA_GRAD_ID, "loss_ssim": LAMBDA_SSIM, "loss_contrast_attention": LAMBDA_CA,
               "loss_contrast_region": LAMBDA_CR, "loss_contrast_edge": LAMBDA_CE}
        bias, coef, coefx = [], [], []
        for name in _G_TERMS:
            row, b, cx = [0.0] * (5 * njobs), 0.0, [0.0] * 4
            parts = terms.items() if name == "loss_G" else [(name, terms[name])]
            for tn, (cf, bb, (x0, x1)) in parts:
                w = lam[tn] if name == "loss_G" else 1.0
                for (j, q), c in cf.items():
                    row[5 * j + q] += w * c
                b += w * bb
                cx[0] += w * x0
                cx[1] += w * x1
            bias.append(b)
            coef.append(row)
            coefx.append(cx)
        return bias, coef, coefx

    def g_step_losses(self, planes, grads):
        """loss_G of trainer.py:469-512 and its terms from the step's planes, plus d(loss_G)/d(plane).

        planes: real_A, real_B, rec_A, rec_B, id_A, id_B, fake_B [N,1,H,W] and dB = D_B(fake_B),
        dA = D_A(fake_A) [N,1,H/16,W/16]; grads: an output tensor for each plane except the two real
        ones (written, not added to).  The batch-coupled ContrastRegion / ContrastEdge terms
        (trainer.py:126-128, 170-180) run their own phases first; every other term is one fused
        launch (ops.gen_loss_fused) that takes their gradients as addends of fake_B's plane.
        Returns a device vector of _G_TERMS values."""
        from .hip import ops
        from .hip.lib import GL_CA, GL_GRAD, GL_L1, GL_MSEC, GL_SSIM
        from .losses import _global
        P = planes
        real_A, real_B, fake_B = P["real_A"], P["real_B"], P["fake_B"]
        cr_m, ce_m = self.criterion_contrast_region, self.criterion_contrast_edge
        if _global(cr_m.global_stats):
            cr_v, cr_g = ops.loss_contrast_region_global(fake_B, real_B, real_A, cr_m.threshold, cr_m.weight,
                                                         parallel.allreduce_sum_, parallel.world())
        else:
            cr_v, cr_g = ops.loss_contrast_region(fake_B, real_B, real_A, cr_m.threshold, cr_m.weight)
        if _global(ce_m.global_stats):
            ce_v, ce_g = ops.loss_contrast_edge_global(fake_B, real_B, parallel.allreduce_sum_, parallel.world())
        else:
            ce_v, ce_g = ops.loss_contrast_edge(fake_B, real_B)
        lc, li = self.lambda_cyc, self.lambda_id
        rec = dict(flags=GL_L1 | GL_GRAD | GL_SSIM, c_l1=lc / 2, c_grad=LAMBDA_GRAD / 2, c_ssim=-LAMBDA_SSIM / 2)
        idt = dict(flags=GL_L1 | GL_GRAD, c_l1=li / 2, c_grad=LAMBDA_GRAD_ID / 2)
        ca_m = self.criterion_contrast_attention
        assert ca_m.blur_kernel == 7, "fused loss: 7x7 contrast-attention box"
        jobs = [dict(pred=P["rec_A"], target=real_A, grad=grads["rec_A"], **rec),
                dict(pred=P["rec_B"], target=real_B, grad=grads["rec_B"], **rec),
                dict(pred=P["id_A"], target=real_A, grad=grads["id_A"], **idt),
                dict(pred=P["id_B"], target=real_B, grad=grads["id_B"], **idt),
                dict(pred=fake_B, target=real_B, source=real_A, grad=grads["fake_B"], flags=GL_CA, c_ca=LAMBDA_CA,
                     add0=cr_g, c_add0=LAMBDA_CR, add1=ce_g, c_add1=LAMBDA_CE),
                dict(pred=P["dB"], grad=grads["dB"], flags=GL_MSEC, c_mse=0.5, t_const=1.0),
                dict(pred=P["dA"], grad=grads["dA"], flags=GL_MSEC, c_mse=0.5, t_const=1.0)]
        return ops.gen_loss_fused(jobs, self._g_loss_recipe(len(jobs)), extra=(cr_v, ce_v),
                                  ssim_data_range=self.criterion_ssim.data_range,
                                  ca=(ca_m.sigma, ca_m.min_weight, ca_m.max_weight))

    def _train_step_explicit(self, real_A, real_B, masks=None):
        """trainer.py:463-525 as an explicit schedule: the Generator / Discriminator forward and
        backward functions of modules/hip/networks.py called directly, every loss term of the G
        step (L1, gradient, SSIM, contrast attention, the GAN MSEs) by one fused loss launch that
        also writes each plane's combined d(loss_G)/d(plane) (modules/hip/ops.py gen_loss_fused),
        the batch-coupled ContrastRegion / ContrastEdge phases first (their gradients enter the
        fused launch as addends), and the input gradients of planes used twice summed by
        in-place adds.  Same math and values as _train_step_autograd."""
        from .hip import networks as net
        from .hip import ops
        from .hip.lib import GL_MSEC
        N = real_A.shape[0]
        G_AB, G_BA, D_A, D_B = self.models
        nb, cb = G_AB.num_residual_blocks, G_AB.use_cbam
        real_A, real_B = real_A.contiguous(), real_B.contiguous()
        mk = (lambda k: torch.cat([masks] * k)) if masks is not None else (lambda k: None)
        pAB = dict(zip(G_AB._keys, [p for _, p in G_AB.named_parameters()]))
        pBA = dict(zip(G_BA._keys, [p for _, p in G_BA.named_parameters()]))
        pDA = [p for _, p in D_A.named_parameters()]
        pDB = [p for _, p in D_B.named_parameters()]

        # --- Generator step (trainer.py:463-514) ---
        ops.range_arena_reset(self.device)  # this step's range records: one zeroing launch
        ops.prepack([p for m in self.models for p in m.parameters()])  # every weight pack of the step, batched
        self.optimizer_G.zero_grad()
        with torch.no_grad():
            ab, S_ab = net.generator_forward(pAB, torch.cat([real_A, real_B]), mk(2), nb, cb, True)
            fake_B, id_B = ab[:N], ab[N:]
            ba, S_ba = net.generator_forward(pBA, torch.cat([real_B, real_A, fake_B]), mk(3), nb, cb, True)
            fake_A, id_A, rec_A = ba[:N], ba[N:2 * N], ba[2 * N:]
            dB, S_dB = net.discriminator_forward(pDB, fake_B, True)
            dA, S_dA = net.discriminator_forward(pDA, fake_A, True)
            rec_B, S_rb = net.generator_forward(pAB, fake_A, masks, nb, cb, True)
            S_ab["out"], S_ba["out"], S_rb["out"] = ab, ba, rec_B
            # every loss term of loss_G, and d(loss_G)/d(plane) written into each plane's slice
            d_ab, d_ba, d_rb = torch.empty_like(ab), torch.empty_like(ba), torch.empty_like(rec_B)
            d_dB, d_dA = torch.empty_like(dB), torch.empty_like(dA)
            vals = self.g_step_losses(
                dict(real_A=real_A, real_B=real_B, rec_A=rec_A, rec_B=rec_B, id_A=id_A, id_B=id_B, fake_B=fake_B,
                     dB=dB, dA=dA),
                dict(rec_A=d_ba[2 * N:], rec_B=d_rb, id_A=d_ba[N:2 * N], id_B=d_ab[N:], fake_B=d_ab[:N],
                     dB=d_dB, dA=d_dA))
            # backward: D input gradients (no D parameter gradients in the G step), then the three
            # Generator calls in reverse; planes with two consumers get the second by an add
            dxB, _ = net.discriminator_backward(S_dB, d_dB, True, False)
            ops.scale_add_(d_ab[:N], dxB.reshape(d_ab[:N].shape))
            dxA, _ = net.discriminator_backward(S_dA, d_dA, True, False)
            # (S_dA / S_dB stay: the D steps below reuse these forwards of the fake samples, the
            # Discriminators' weights being unchanged until their own steps)
            dx_rb, _ = net.generator_backward(S_rb, d_rb, True, 1, 0, pAB)
            torch.add(dxA.reshape(d_ba[:N].shape), dx_rb.reshape(d_ba[:N].shape), out=d_ba[:N])
            del S_rb, dxA, dx_rb
            dx_ba, _ = net.generator_backward(S_ba, d_ba, True, 1, 2 * N, pBA, slice_only=True)
            ops.scale_add_(d_ab[:N], dx_ba.reshape(d_ab[:N].shape))
            del S_ba, dx_ba
            net.generator_backward(S_ab, d_ab, False, 1, 0, pAB)
            del S_ab
        parallel.allreduce_mean_(self.optimizer_G.flat_g)  # replica mean of the G gradient (one all-reduce)
        self.optimizer_G.step()
        out = {k: vals[i] for i, k in enumerate(_G_TERMS)}

        # --- Discriminator steps (trainer.py:517-525) ---
        # D(fake.detach()) is the forward the G step already ran on the same samples with the same
        # Discriminator weights (only G moved since): its outputs and saved activations are reused,
        # and only D(real) is computed here.  The weight gradient is the real half's backward plus
        # the fake half's (the second one added into .grad).
        for name, D, params, real, o_f, S_f in (("loss_D_A", D_A, pDA, real_A, dA, S_dA),
                                                ("loss_D_B", D_B, pDB, real_B, dB, S_dB)):
            opt = self.optimizer_D_A if D is D_A else self.optimizer_D_B
            opt.zero_grad()
            with torch.no_grad():
                o_r, S_r = net.discriminator_forward(params, real, True)
                d_r, d_f = torch.empty_like(o_r), torch.empty_like(o_f)
                jobs = [dict(pred=o_r, grad=d_r, flags=GL_MSEC, c_mse=0.5, t_const=1.0),
                        dict(pred=o_f, grad=d_f, flags=GL_MSEC, c_mse=0.5, t_const=0.0)]
                v = ops.gen_loss_fused(jobs, ([0.0], [[0, 0, 0, 0, .5, 0, 0, 0, 0, .5]], [[0.0] * 4]))
                pd = dict(enumerate(params))
                net.discriminator_backward(S_r, d_r, False, True, pd)
                net.discriminator_backward(S_f, d_f, False, True, pd)
                del S_r
            parallel.allreduce_mean_(opt.flat_g)
            opt.step()
            out[name] = v[0]
        del S_dA, S_dB
        return out

    def _train_step_autograd(self, real_A, real_B, masks=None):
        """The same step on the autograd Functions (modules/hip/networks.py) and loss modules."""
        N = real_A.shape[0]
        G_AB, G_BA, D_A, D_B = self.models
        mk = (lambda k: torch.cat([masks] * k)) if masks is not None else (lambda k: None)

        # --- Generator step (trainer.py:463-514) ---
        # Three Generator launches instead of the reference's six calls: G_A2B on
        # [real_A; real_B] -> [fake_B; id_B]; G_B2A on [real_B; real_A; fake_B] ->
        # [fake_A; id_A; rec_A]; G_A2B on fake_A -> rec_B.  Same inputs and weights per sample
        # as trainer.py:466-481 (InstanceNorm is per sample), fewer and fuller launches.
        self.optimizer_G.zero_grad()
        ab = G_AB(torch.cat([real_A, real_B]), mk(2))              # [fake_B ; id_B]
        fake_B, id_B = ab[:N], ab[N:]
        ba = G_BA(torch.cat([real_B, real_A, fake_B]), mk(3),      # [fake_A ; id_A ; rec_A]
                  input_grad_from=2 * N)                          # only fake_B needs dL/dx
        fake_A, id_A, rec_A = ba[:N], ba[N:2 * N], ba[2 * N:]
        loss_id = (self.criterion_identity(id_A, real_A) + self.criterion_identity(id_B, real_B)) / 2
        loss_GAN = (self.criterion_GAN(D_B(fake_B, params_require_grad=False), 1.0)
                    + self.criterion_GAN(D_A(fake_A, params_require_grad=False), 1.0)) / 2
        rec_B = G_AB(fake_A, masks)
        loss_cycle = (self.criterion_cycle(rec_A, real_A) + self.criterion_cycle(rec_B, real_B)) / 2
        loss_grad_cycle = (self.criterion_gradient(rec_A, real_A) + self.criterion_gradient(rec_B, real_B)) / 2
        loss_grad_id = (self.criterion_gradient(id_A, real_A) + self.criterion_gradient(id_B, real_B)) / 2
        loss_ssim = 1 - ((self.criterion_ssim(rec_A, real_A) + self.criterion_ssim(rec_B, real_B)) / 2)
        loss_ca = self.criterion_contrast_attention(fake_B, real_B, real_A)
        loss_cr = self.criterion_contrast_region(fake_B, real_B, real_A)
        loss_ce = self.criterion_contrast_edge(fake_B, real_B, real_A)
        loss_G = (loss_GAN + self.lambda_cyc * loss_cycle + self.lambda_id * loss_id
                  + LAMBDA_GRAD * loss_grad_cycle + LAMBDA_GRAD_ID * loss_grad_id + LAMBDA_SSIM * loss_ssim
                  + LAMBDA_CA * loss_ca + LAMBDA_CR * loss_cr + LAMBDA_CE * loss_ce)
        loss_G.backward()
        parallel.allreduce_mean_(self.optimizer_G.flat_g)  # replica mean of the G gradient
        self.optimizer_G.step()

        # --- Discriminator steps (trainer.py:517-525), real and fake batched ---
        self.optimizer_D_A.zero_grad()
        outA = D_A(torch.cat([real_A, fake_A.detach()]))
        loss_D_A = (self.criterion_GAN(outA[:N], 1.0) + self.criterion_GAN(outA[N:], 0.0)) / 2
        loss_D_A.backward()
        parallel.allreduce_mean_(self.optimizer_D_A.flat_g)
        self.optimizer_D_A.step()

        self.optimizer_D_B.zero_grad()
        outB = D_B(torch.cat([real_B, fake_B.detach()]))
        loss_D_B = (self.criterion_GAN(outB[:N], 1.0) + self.criterion_GAN(outB[N:], 0.0)) / 2
        loss_D_B.backward()
        parallel.allreduce_mean_(self.optimizer_D_B.flat_g)
        self.optimizer_D_B.step()

        return {"loss_G": loss_G.detach(), "loss_GAN": loss_GAN.detach(), "loss_cycle": loss_cycle.detach(),
                "loss_id": loss_id.detach(), "loss_grad_cycle": loss_grad_cycle.detach(),
                "loss_grad_id": loss_grad_id.detach(), "loss_ssim": loss_ssim.detach(),
                "loss_contrast_attention": loss_ca.detach(), "loss_contrast_region": loss_cr.detach(),
                "loss_contrast_edge": loss_ce.detach(), "loss_D_A": loss_D_A.detach(),
                "loss_D_B": loss_D_B.detach()}

    @torch.no_grad()
    def validation_loss(self, real_A, real_B, masks=None):
        """trainer.py:227-248: GAN + lambda_cyc * cycle + lambda_id * identity."""
        fake_B, fake_A = self.G_A2B(real_A, masks), self.G_B2A(real_B, masks)
        rec_A, rec_B = self.G_B2A(fake_B, masks), self.G_A2B(fake_A, masks)
        id_A, id_B = self.G_B2A(real_A, masks), self.G_A2B(real_B, masks)
        loss_id = (self.criterion_identity(id_A, real_A) + self.criterion_identity(id_B, real_B)) / 2
        loss_GAN = (self.criterion_GAN(self.D_B(fake_B), 1.0) + self.criterion_GAN(self.D_A(fake_A), 1.0)) / 2
        loss_cycle = (self.criterion_cycle(rec_A, real_A) + self.criterion_cycle(rec_B, real_B)) / 2
        return loss_GAN + self.lambda_cyc * loss_cycle + self.lambda_id * loss_id


class ConcurrentCycleGANs:
    """Several CycleGANSystems trained in the same process (BASELINE config 5: the soft-tissue
    (cin 3) and lung (cin 2) models; the reference trains them one after the other,
    train.py:27-38): each step runs the systems one after the other on the caller's stream.

    A two-stream schedule (one HIP stream per model, each on its own compute-unit partition) was
    built and measured in rounds 1-3: 1.8 % faster than this one (32.77 vs 32.19 img/s, f16x3) and
    exact only with pair-aligned CU partitions, because streams whose waves share a compute-unit
    pair sometimes gave wrong results (Config 5).  It is not part of the product.
    On 8 GPUs config 5 runs as split GPU groups (bench.py --dual-schedule groups,
    modules/parallel.py split_groups): each model on its own half of the ranks."""

    def __init__(self, systems, device, schedule="serial"):
        if schedule != "serial":
            raise ValueError("ConcurrentCycleGANs: the only schedule is 'serial' (DESIGN.md §3, Config 5)")
        self.systems = list(systems)
        self.device = torch.device(device)
        self.schedule = schedule

    def train_step(self, batches):
        """batches: one (real_A, real_B, masks) per system.  Returns one loss dict per system
        (device tensors)."""
        return [sysm.train_step(*b) for sysm, b in zip(self.systems, batches)]


# -------------------------------------------------------------------------------------------
# data: a DICOM tree (modules/dataset.py: decode on the loader workers, HU transform + masks on
# the GPU) when data_root/dataset_names exists, synthetic slices of the reference's shapes
# otherwise (or with --synthetic).
# -------------------------------------------------------------------------------------------
class SyntheticSlices(torch.utils.data.Dataset):
    """Deterministic synthetic slices: A, B ~ U(-1,1) [1,H,W], masks ~ Bernoulli(0.3)."""

    def __init__(self, n, img_size, n_masks, seed=0):
        self.n, self.img_size, self.n_masks, self.seed = n, img_size, n_masks, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        s = self.img_size
        out = {"A": torch.rand(1, s, s, generator=g) * 2 - 1, "B": torch.rand(1, s, s, generator=g) * 2 - 1}
        if self.n_masks:
            out["masks"] = (torch.rand(self.n_masks, s, s, generator=g) < 0.3).float()
        return out


def _to_dev(batch, device, prep=None):
    """Batch -> (real_A, real_B, masks) on the device; decoded DICOM batches go through the
    GPU preprocessor (HU transform + masks, modules/dataset.py)."""
    if prep is not None and (isinstance(batch, list) or "A_raw" in batch):
        batch = prep(batch)
    real_A = batch["A"].to(device, non_blocking=True)
    real_B = batch["B"].to(device, non_blocking=True)
    masks = batch["masks"].to(device, non_blocking=True) if "masks" in batch else None
    return real_A, real_B, masks


def validate_and_save_images(epoch, system, val_loader, args, device, fixed_val_batch, prep=None):
    """trainer.py:187-294: mean validation G loss over the (rank-sharded) validation set and an
    [NCCT | fake CECT | CECT] windowed image grid of a fixed batch (rank 0)."""
    for m in system.models:
        m.eval()
    total = torch.zeros((), device=device)
    count = 0
    for batch in val_loader:
        real_A, real_B, masks = _to_dev(batch, device, prep)
        total += system.validation_loss(real_A, real_B, masks)
        count += 1
    stats = torch.stack([total, torch.tensor(float(count), device=device)])
    if parallel.world() > 1:
        torch.distributed.all_reduce(stats)
    avg = float(stats[0] / max(float(stats[1]), 1.0))
    if parallel.rank() == 0 and fixed_val_batch is not None:
        try:
            with torch.no_grad():
                real_A, real_B, masks = _to_dev(fixed_val_batch, device, prep)
                fake_B = system.G_A2B(real_A, masks)
                grid = torch.cat((apply_windowing(real_A, args), apply_windowing(fake_B, args),
                                  apply_windowing(real_B, args)), -1)
            _save_grid(grid, os.path.join(args.training_dir, "images", f"epoch_{epoch + 1}.jpg"),
                       nrow=min(real_A.size(0), 4))
        except Exception as e:  # the reference also swallows preview failures (trainer.py:284)
            print(f"Warning: Failed to save sample images: {e}")
    for m in system.models:
        m.train()
    return avg


def _save_grid(grid, path, nrow):
    from PIL import Image
    g = grid.detach().float().clamp(0, 1).cpu()
    n, _, h, w = g.shape
    rows = math.ceil(n / nrow)
    canvas = torch.zeros(rows * (h + 2) + 2, nrow * (w + 2) + 2)
    for i in range(n):
        r, c = divmod(i, nrow)
        canvas[2 + r * (h + 2): 2 + r * (h + 2) + h, 2 + c * (w + 2): 2 + c * (w + 2) + w] = g[i, 0]
    Image.fromarray((canvas * 255 + 0.5).clamp(0, 255).byte().numpy(), mode="L").save(path)


def _build_datasets(args, n_masks):
    """Patient-level split of trainer.py:422-430 when a DICOM dataset is available; synthetic
    slices otherwise (or with --synthetic)."""
    if not getattr(args, "synthetic", False):
        root = os.path.join(args.data_root, args.dataset_names)
        if os.path.isdir(root):
            from .dataset import DicomDataset
            dirs = sorted(glob.glob(os.path.join(root, "*")))
            random.seed(42)
            random.shuffle(dirs)
            vc = int(len(dirs) * args.val_split)
            return DicomDataset(dirs[vc:], args), DicomDataset(dirs[:vc], args)
    n = int(getattr(args, "synthetic_slices", 64))
    nv = max(int(n * args.val_split), 1)
    return (SyntheticSlices(n, args.img_size, n_masks, seed=1),
            SyntheticSlices(nv, args.img_size, n_masks, seed=2))


def train_cycle_gan(args, target_range):
    """trainer.py:297-597 (one process per GPU; args.batch_size is the GLOBAL batch, as in the
    reference, split evenly over ranks)."""
    if target_range not in ["soft_tissue", "lung"]:
        raise ValueError("target_range must be either 'soft_tissue' or 'lung'")
    rank, world, local = parallel.init_from_env()
    if not torch.cuda.is_available():
        raise RuntimeError("train_cycle_gan runs on the MI355X kernels; no GPU is visible")
    device = torch.device(f"cuda:{local}")
    torch.cuda.set_device(device)

    cur = os.path.join(args.training_dir, target_range)
    args.training_dir = cur
    images_dir = os.path.join(cur, "images")
    saved_models_dir = os.path.join(cur, "saved_models")
    if rank == 0:
        os.makedirs(images_dir, exist_ok=True)
        os.makedirs(saved_models_dir, exist_ok=True)
        print(f"Starting training with args: {args}")

    input_channels = 1
    n_masks = 0
    if getattr(args, "use_masks", False) and getattr(args, "mask_folders", []):
        n_masks = len(args.mask_folders)
        input_channels = 1 + n_masks
    use_cbam = getattr(args, "use_cbam", True)
    nb = int(getattr(args, "num_residual_blocks", 9))
    torch.manual_seed(int(getattr(args, "seed", 0)))
    from . import losses as _losses
    _losses.GLOBAL_STATS = False if getattr(args, "per_rank_loss_stats", False) else None
    if rank == 0:
        print(f"Batch-coupled loss statistics (ContrastRegion/ContrastEdge): {_losses.stats_mode()}")
    system = CycleGANSystem(input_channels, nb, use_cbam, lr=args.lr, lambda_cyc=args.lambda_cyc,
                            lambda_id=args.lambda_id, device=device)
    lr_lambda = lambda epoch: 1.0 - max(0, epoch + 1 - args.decay_epoch) / (args.epochs - args.decay_epoch)
    schedulers = [torch.optim.lr_scheduler.LambdaLR(o, lr_lambda) for o in system.optimizers]

    start_epoch, best_val_loss, best_epoch = 0, float("inf"), -1
    ckpt_path = os.path.join(saved_models_dir, args.resume) if args.resume else None
    if ckpt_path and os.path.isfile(ckpt_path):
        print(f"=> Loading checkpoint '{ckpt_path}'")
        start_epoch, best_val_loss, best_epoch = _load_checkpoint(ckpt_path, system, schedulers, device)
    elif ckpt_path:
        print(f"=> No checkpoint found at '{ckpt_path}'")

    train_ds, val_ds = _build_datasets(args, n_masks)
    if args.batch_size % world:
        raise ValueError(f"--batch_size {args.batch_size} (the global batch, as in the reference) must be a "
                         f"multiple of the {world} processes")
    per_rank = args.batch_size // world
    tsampler = torch.utils.data.DistributedSampler(train_ds, world, rank, shuffle=True) if world > 1 else None
    vsampler = torch.utils.data.DistributedSampler(val_ds, world, rank, shuffle=False) if world > 1 else None
    nw = min(int(getattr(args, "num_workers", 0)), 16)
    prep, collate_fn = None, None
    if not isinstance(train_ds, SyntheticSlices):
        from .dataset import SliceBatchPreprocessor, collate
        prep, collate_fn = SliceBatchPreprocessor(args, device), collate
    dl = torch.utils.data.DataLoader(train_ds, batch_size=per_rank, shuffle=tsampler is None, sampler=tsampler,
                                     num_workers=nw, pin_memory=True, drop_last=world > 1,
                                     persistent_workers=nw > 0, collate_fn=collate_fn)
    vdl = torch.utils.data.DataLoader(val_ds, batch_size=per_rank * 2, shuffle=False, sampler=vsampler,
                                      num_workers=nw, pin_memory=True, collate_fn=collate_fn)
    if len(dl) == 0:
        raise ValueError(f"no training batches: {len(train_ds)} slices for {world} processes x batch {per_rank}")
    fixed_val_batch = next(iter(vdl))
    if rank == 0:
        print(f"Train/Val split: {len(train_ds)} slices / {len(val_ds)} slices")

    max_steps = int(getattr(args, "max_steps_per_epoch", 0) or 0)
    for epoch in range(start_epoch, args.epochs):
        if tsampler is not None:
            tsampler.set_epoch(epoch)
        system.train()
        t0 = time.time()
        for i, batch in enumerate(dl):
            real_A, real_B, masks = _to_dev(batch, device, prep)
            losses = system.train_step(real_A, real_B, masks)
            if rank == 0 and (i % max(int(getattr(args, "log_every", 10)), 1) == 0):
                print(f"Epoch {epoch + 1}/{args.epochs} step {i}: G_loss {float(losses['loss_G']):.4f} "
                      f"D_loss {float(losses['loss_D_A'] + losses['loss_D_B']):.4f} contrast "
                      f"{float(losses['loss_contrast_attention'] + losses['loss_contrast_region'] + losses['loss_contrast_edge']):.4f}",
                      flush=True)
            if max_steps and i + 1 >= max_steps:
                break
        for s in schedulers:
            s.step()
        torch.cuda.synchronize()
        val_loss = validate_and_save_images(epoch, system, vdl, args, device, fixed_val_batch, prep)
        if rank == 0:
            print(f"\nEpoch {epoch + 1} finished in {time.time() - t0:.1f}s. Validation Generator Loss: {val_loss:.4f}")
            _save_epoch(system, schedulers, args, saved_models_dir, epoch, val_loss, best_val_loss, best_epoch)
        if val_loss < best_val_loss:
            best_val_loss, best_epoch = val_loss, epoch + 1
    return system


def _load_checkpoint(path, system, schedulers, device):
    """Resume from checkpoint.pth.tar (trainer.py:374-405 layout).  The file pickles the args
    Namespace (trainer.py:594); it is read with the weights-only unpickler with
    argparse.Namespace allow-listed, so loading never executes code from the file.  Accepts
    the reference's DataParallel ``module.``-prefixed state_dicts.  Returns
    (start_epoch, best_val_loss, best_epoch)."""
    import argparse
    with torch.serialization.safe_globals([argparse.Namespace]):
        ck = torch.load(path, map_location=device, weights_only=True)
    for key, m in zip(("G_A2B", "G_B2A", "D_A", "D_B"), system.models):
        sd = ck[f"{key}_state_dict"]
        if all(k.startswith("module.") for k in sd):
            sd = {k[len("module."):]: v for k, v in sd.items()}
        m.load_state_dict(sd)
    for key, o in zip(("G", "D_A", "D_B"), system.optimizers):
        o.load_state_dict(ck[f"optimizer_{key}_state_dict"])
    for key, s in zip(("G", "D_A", "D_B"), schedulers):
        s.load_state_dict(ck[f"scheduler_{key}_state_dict"])
    return ck["epoch"] + 1, ck.get("best_val_loss", float("inf")), ck.get("best_epoch", -1)


def _save_epoch(system, schedulers, args, saved_models_dir, epoch, val_loss, best_val_loss, best_epoch):
    """trainer.py:549-597 — identical file names and checkpoint keys."""
    G_A2B, G_B2A, D_A, D_B = system.models
    if val_loss < best_val_loss:
        if best_epoch != -1:
            for nm in ("G_A2B", "G_B2A"):
                old = os.path.join(saved_models_dir, f"{nm}_best_epoch_{best_epoch}.pth")
                if os.path.exists(old):
                    os.remove(old)
        best_val_loss, best_epoch = val_loss, epoch + 1
        torch.save(G_A2B.state_dict(), os.path.join(saved_models_dir, f"G_A2B_best_epoch_{best_epoch}.pth"))
        torch.save(G_B2A.state_dict(), os.path.join(saved_models_dir, f"G_B2A_best_epoch_{best_epoch}.pth"))
        print(f"New best models saved for epoch {best_epoch} with validation loss: {best_val_loss:.4f}")
    torch.save(G_A2B.state_dict(), os.path.join(saved_models_dir, f"G_A2B_epoch_{epoch + 1}.pth"))
    torch.save(G_B2A.state_dict(), os.path.join(saved_models_dir, f"G_B2A_epoch_{epoch + 1}.pth"))
    torch.save(G_A2B.state_dict(), os.path.join(saved_models_dir, "G_A2B_last.pth"))
    torch.save(G_B2A.state_dict(), os.path.join(saved_models_dir, "G_B2A_last.pth"))
    state = {
        "epoch": epoch,
        "G_A2B_state_dict": G_A2B.state_dict(), "G_B2A_state_dict": G_B2A.state_dict(),
        "D_A_state_dict": D_A.state_dict(), "D_B_state_dict": D_B.state_dict(),
        "optimizer_G_state_dict": system.optimizer_G.state_dict(),
        "optimizer_D_A_state_dict": system.optimizer_D_A.state_dict(),
        "optimizer_D_B_state_dict": system.optimizer_D_B.state_dict(),
        "scheduler_G_state_dict": schedulers[0].state_dict(),
        "scheduler_D_A_state_dict": schedulers[1].state_dict(),
        "scheduler_D_B_state_dict": schedulers[2].state_dict(),
        "best_val_loss": best_val_loss, "best_epoch": best_epoch, "args": args,
    }
    torch.save(state, os.path.join(saved_models_dir, "checkpoint.pth.tar"))
    print(f"Checkpoint and last models saved for epoch {epoch + 1}.\n")
