"""CPU fp32 restatement of the DuCoSy-GAN CycleGAN training hot path (the ORACLE).

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module.  It is the checker,
never the thing measured or shipped: the product path (``ducosy-gan_amd/``) runs
the hand-written HIP kernels and fails loudly without them.

Written functionally (parameter dicts keyed by the reference's state_dict names,
``torch.nn.functional`` calls) so it is a restatement, not a copy.  Each function
cites the reference file:line it follows (paths relative to the reference repo).

Pinning: ``tests/test_oracle_golden.py`` checks every function here against the
golden vectors in ``tests/golden/`` which ``tests/golden/make_golden.py`` produced
by importing the reference itself in the build container.  SSIM is the exception:
``pytorch_msssim`` (unpinned in requirements.txt:27) is not installed and not in
the reference tree, so ``ssim`` below restates its published algorithm and is
**parity unpinned** (the golden step fixtures use this same restatement as the
reference's SSIM stand-in).
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence

import torch
import torch.nn.functional as F

Params = Dict[str, torch.Tensor]

IN_EPS = 1e-5  # nn.InstanceNorm2d default eps (modules/model.py:61,94)


# ---------------------------------------------------------------------------
# parameter layouts (state_dict key order == .parameters() order)
# ---------------------------------------------------------------------------
def generator_param_shapes(input_channels: int = 1, num_residual_blocks: int = 9,
                           use_cbam: bool = True) -> Dict[str, tuple]:
    """Keys/shapes of modules/model.py:90-113 Generator.state_dict()."""
    s: Dict[str, tuple] = {}
    s["model.1.weight"] = (64, input_channels, 7, 7)
    s["model.1.bias"] = (64,)
    s["model.4.weight"] = (128, 64, 3, 3)
    s["model.4.bias"] = (128,)
    s["model.7.weight"] = (256, 128, 3, 3)
    s["model.7.bias"] = (256,)
    for b in range(num_residual_blocks):
        p = f"model.{10 + b}"
        s[f"{p}.block.1.weight"] = (256, 256, 3, 3)
        s[f"{p}.block.1.bias"] = (256,)
        s[f"{p}.block.5.weight"] = (256, 256, 3, 3)
        s[f"{p}.block.5.bias"] = (256,)
        if use_cbam:
            s[f"{p}.cbam.channel_attention.fc.0.weight"] = (16, 256, 1, 1)
            s[f"{p}.cbam.channel_attention.fc.2.weight"] = (256, 16, 1, 1)
            s[f"{p}.cbam.spatial_attention.conv.weight"] = (1, 2, 7, 7)
    u = 10 + num_residual_blocks
    s[f"model.{u + 1}.weight"] = (128, 256, 3, 3)
    s[f"model.{u + 1}.bias"] = (128,)
    s[f"model.{u + 5}.weight"] = (64, 128, 3, 3)
    s[f"model.{u + 5}.bias"] = (64,)
    s[f"model.{u + 9}.weight"] = (1, 64, 7, 7)
    s[f"model.{u + 9}.bias"] = (1,)
    return s


def discriminator_param_shapes(input_channels: int = 1) -> Dict[str, tuple]:
    """Keys/shapes of modules/model.py:118-131 Discriminator.state_dict()."""
    return {
        "model.0.weight": (64, input_channels, 4, 4), "model.0.bias": (64,),
        "model.2.weight": (128, 64, 4, 4), "model.2.bias": (128,),
        "model.5.weight": (256, 128, 4, 4), "model.5.bias": (256,),
        "model.8.weight": (512, 256, 4, 4), "model.8.bias": (512,),
        "model.12.weight": (1, 512, 4, 4), "model.12.bias": (1,),
    }


# ---------------------------------------------------------------------------
# networks
# ---------------------------------------------------------------------------
def _inorm(x: torch.Tensor) -> torch.Tensor:
    # nn.InstanceNorm2d(affine=False, track_running_stats=False): per-(n,c) batch stats,
    # biased variance, eps 1e-5.
    return F.instance_norm(x, eps=IN_EPS)


def channel_attention(p: Params, prefix: str, x: torch.Tensor) -> torch.Tensor:
    """modules/model.py:6-24: shared 1x1 MLP on avg- and max-pooled planes, sigmoid gate."""
    w1 = p[f"{prefix}.fc.0.weight"]
    w2 = p[f"{prefix}.fc.2.weight"]

    def mlp(v):
        return F.conv2d(F.relu(F.conv2d(v, w1)), w2)

    avg = x.mean(dim=(2, 3), keepdim=True)
    mx = F.adaptive_max_pool2d(x, 1)  # gradient to the argmax element, as nn.AdaptiveMaxPool2d
    return x * torch.sigmoid(mlp(avg) + mlp(mx))


def spatial_attention(p: Params, prefix: str, x: torch.Tensor) -> torch.Tensor:
    """modules/model.py:27-39: [mean_c, max_c] -> 7x7 conv (zero pad 3, no bias) -> sigmoid."""
    w = p[f"{prefix}.conv.weight"]
    k = w.shape[-1]
    s = torch.cat([x.mean(dim=1, keepdim=True), x.max(dim=1, keepdim=True)[0]], dim=1)
    return x * torch.sigmoid(F.conv2d(s, w, padding=k // 2))


def residual_block(p: Params, prefix: str, x: torch.Tensor, use_cbam: bool = True) -> torch.Tensor:
    """modules/model.py:56-87 (ResidualBlock / ResidualBlockWithCBAM)."""
    h = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"),
                 p[f"{prefix}.block.1.weight"], p[f"{prefix}.block.1.bias"])
    h = F.relu(_inorm(h))
    h = F.conv2d(F.pad(h, (1, 1, 1, 1), mode="reflect"),
                 p[f"{prefix}.block.5.weight"], p[f"{prefix}.block.5.bias"])
    h = _inorm(h)
    if use_cbam:
        h = channel_attention(p, f"{prefix}.cbam.channel_attention", h)
        h = spatial_attention(p, f"{prefix}.cbam.spatial_attention", h)
    return x + h


def generator_stages(p: Params, x: torch.Tensor, num_residual_blocks: int = 9,
                     use_cbam: bool = True) -> Dict[str, torch.Tensor]:
    """modules/model.py:90-115 Generator.forward (ResNet-CBAM, output 1 channel, tanh), returning
    every stage's activation: "stem", "down1", "down2" (conv + IN + ReLU), "res{b}" (each residual
    block's output), "up1", "up2" and "out"."""
    st = {}
    h = F.conv2d(F.pad(x, (3, 3, 3, 3), mode="reflect"), p["model.1.weight"], p["model.1.bias"])
    h = st["stem"] = F.relu(_inorm(h))
    for name, idx in (("down1", 4), ("down2", 7)):  # stride-2, zero pad 1 (modules/model.py:96-98)
        h = F.conv2d(h, p[f"model.{idx}.weight"], p[f"model.{idx}.bias"], stride=2, padding=1)
        h = st[name] = F.relu(_inorm(h))
    for b in range(num_residual_blocks):
        h = st[f"res{b}"] = residual_block(p, f"model.{10 + b}", h, use_cbam)
    u = 10 + num_residual_blocks
    for name, idx in (("up1", u + 1), ("up2", u + 5)):  # nearest x2 upsample, conv zero pad 1 (:107-111)
        h = F.interpolate(h, scale_factor=2, mode="nearest")
        h = F.conv2d(h, p[f"model.{idx}.weight"], p[f"model.{idx}.bias"], padding=1)
        h = st[name] = F.relu(_inorm(h))
    h = F.conv2d(F.pad(h, (3, 3, 3, 3), mode="reflect"),
                 p[f"model.{u + 9}.weight"], p[f"model.{u + 9}.bias"])
    st["out"] = torch.tanh(h)
    return st


def generator_forward(p: Params, x: torch.Tensor, num_residual_blocks: int = 9,
                      use_cbam: bool = True) -> torch.Tensor:
    """modules/model.py:90-115 Generator.forward (ResNet-CBAM, output 1 channel, tanh)."""
    return generator_stages(p, x, num_residual_blocks, use_cbam)["out"]


def discriminator_forward(p: Params, x: torch.Tensor) -> torch.Tensor:
    """modules/model.py:118-131 PatchGAN: C4s2 x4 (IN on all but the first), LReLU 0.2,
    ZeroPad2d((1,0,1,0)), C4 p1 -> 1 channel."""
    h = F.leaky_relu(F.conv2d(x, p["model.0.weight"], p["model.0.bias"], stride=2, padding=1), 0.2)
    for idx in (2, 5, 8):
        h = F.conv2d(h, p[f"model.{idx}.weight"], p[f"model.{idx}.bias"], stride=2, padding=1)
        h = F.leaky_relu(_inorm(h), 0.2)
    h = F.pad(h, (1, 0, 1, 0))
    return F.conv2d(h, p["model.12.weight"], p["model.12.bias"], padding=1)


# ---------------------------------------------------------------------------
# losses (modules/trainer.py:22-184, :347-358) and SSIM (pytorch_msssim restated)
# ---------------------------------------------------------------------------
def l1(a, b):
    return (a - b).abs().mean()  # nn.L1Loss (trainer.py:348-349)


def mse(a, b):
    return ((a - b) ** 2).mean()  # nn.MSELoss (trainer.py:347)


def gradient_loss(pred, target):
    """modules/trainer.py:22-40: separate means over the H- and W-difference maps."""
    dyp = (pred[:, :, 1:, :] - pred[:, :, :-1, :]).abs()
    dyt = (target[:, :, 1:, :] - target[:, :, :-1, :]).abs()
    dxp = (pred[:, :, :, 1:] - pred[:, :, :, :-1]).abs()
    dxt = (target[:, :, :, 1:] - target[:, :, :, :-1]).abs()
    return (dxp - dxt).abs().mean() + (dyp - dyt).abs().mean()


def _box(x, k):
    # nn.AvgPool2d(k, stride=1, padding=k//2), count_include_pad=True
    return F.avg_pool2d(x, k, stride=1, padding=k // 2, count_include_pad=True)


def contrast_attention_loss(pred, target, source, sigma=0.1, min_weight=1.0, max_weight=3.0,
                            blur_kernel=5):
    """modules/trainer.py:43-86 (instantiated sigma=.15, k=7 at :356)."""
    tb, sb, pb = _box(target, blur_kernel), _box(source, blur_kernel), _box(pred, blur_kernel)
    w = min_weight + (max_weight - min_weight) * (1.0 - torch.exp(-(tb - sb).abs() / sigma))
    return (w * (pb - tb).abs()).mean()


def contrast_region_loss(pred, target, source, threshold=0.3, weight=2.0):
    """modules/trainer.py:89-130 (instantiated threshold=.15, weight=1.5 at :357).
    Global mean/std are over the whole batch tensor; std is unbiased."""
    pp, tp, sp = F.avg_pool2d(pred, 8, 8), F.avg_pool2d(target, 8, 8), F.avg_pool2d(source, 8, 8)
    m = torch.sigmoid(5.0 * ((tp - sp) - threshold))
    region = (m * (pp - tp).abs()).mean()
    dist = (pred.mean() - target.mean()).abs() + (pred.std() - target.std()).abs()
    return weight * (region + 0.5 * dist)


_SOBEL_X = torch.tensor([[-1.0, 0.0, 1.0], [-2.0, 0.0, 2.0], [-1.0, 0.0, 1.0]]).view(1, 1, 3, 3)
_SOBEL_Y = torch.tensor([[-1.0, -2.0, -1.0], [0.0, 0.0, 0.0], [1.0, 2.0, 1.0]]).view(1, 1, 3, 3)


def edges(img):
    """modules/trainer.py:150-155: Sobel magnitude with eps 1e-6, zero pad 1."""
    ex = F.conv2d(img, _SOBEL_X.to(img), padding=1)
    ey = F.conv2d(img, _SOBEL_Y.to(img), padding=1)
    return torch.sqrt(ex ** 2 + ey ** 2 + 1e-6)


def contrast_edge_loss(pred, target, source=None):
    """modules/trainer.py:157-184: |d mean| + |d std(unbiased)| + |d mean(top 10%)| of edge maps,
    statistics over the whole batch tensor, k = int(0.1 * numel)."""
    pe, te = edges(pred), edges(target)
    stats = (pe.mean() - te.mean()).abs() + (pe.std() - te.std()).abs()
    k = int(pe.numel() * 0.1)
    ptop = torch.topk(pe.flatten(), k).values.mean()
    ttop = torch.topk(te.flatten(), k).values.mean()
    return stats + (ptop - ttop).abs()


def gauss_window_1d(size: int = 11, sigma: float = 1.5) -> torch.Tensor:
    """pytorch_msssim._fspecial_gauss_1d: normalised 1-d gaussian, float32."""
    c = torch.arange(size, dtype=torch.float32) - (size // 2)
    g = torch.exp(-(c ** 2) / (2 * sigma ** 2))
    return g / g.sum()


def ssim(X, Y, data_range: float = 1.0, win_size: int = 11, win_sigma: float = 1.5,
         K=(0.01, 0.03)):
    """pytorch_msssim.ssim(size_average=True) restated [PARITY UNPINNED]: separable VALID
    gaussian filtering (H pass then W pass), C1=(K1*R)^2, C2=(K2*R)^2, mean of ssim_map per
    (n, c) then over everything.  Used at modules/trainer.py:351,485 with data_range=1."""
    C = X.shape[1]
    g = gauss_window_1d(win_size, win_sigma).to(X)
    wh = g.view(1, 1, win_size, 1).repeat(C, 1, 1, 1)
    ww = g.view(1, 1, 1, win_size).repeat(C, 1, 1, 1)

    def filt(t):
        return F.conv2d(F.conv2d(t, wh, groups=C), ww, groups=C)

    C1 = (K[0] * data_range) ** 2
    C2 = (K[1] * data_range) ** 2
    mu1, mu2 = filt(X), filt(Y)
    s11 = filt(X * X) - mu1 * mu1
    s22 = filt(Y * Y) - mu2 * mu2
    s12 = filt(X * Y) - mu1 * mu2
    cs = (2 * s12 + C2) / (s11 + s22 + C2)
    smap = ((2 * mu1 * mu2 + C1) / (mu1 * mu1 + mu2 * mu2 + C1)) * cs
    return smap.flatten(2).mean(-1).mean()


# ---------------------------------------------------------------------------
# the training step (modules/trainer.py:447-525)
# ---------------------------------------------------------------------------
LAMBDA_GRAD, LAMBDA_GRAD_ID, LAMBDA_SSIM = 5.0, 2.5, 2.0          # trainer.py:493-495
LAMBDA_CA, LAMBDA_CR, LAMBDA_CE = 2.0, 1.5, 1.0                    # trainer.py:500-502


def g_loss_terms(real_A, real_B, rec_A, rec_B, id_A, id_B, fake_B, dB, dA, lambda_cyc=10.0,
                 lambda_id=5.0, loss_GAN=None) -> Dict[str, torch.Tensor]:
    """loss_G of modules/trainer.py:469-512 and its nine terms from the step's planes (id, cycle
    and fake images [N,1,H,W]; dB = D_B(fake_B), dA = D_A(fake_A) [N,1,H/16,W/16]).  loss_id is
    trainer.py:474-476, loss_GAN :477-480 (labels of ones, :459), loss_cycle :485-487, the
    gradient terms :490-492, SSIM :494-496, the contrast terms :498-502 (instantiated :356-358).
    ``loss_GAN`` given: use it instead of the MSE of dB / dA."""
    loss_id = (l1(id_A, real_A) + l1(id_B, real_B)) / 2
    if loss_GAN is None:
        loss_GAN = (mse(dB, torch.ones_like(dB)) + mse(dA, torch.ones_like(dA))) / 2
    loss_cycle = (l1(rec_A, real_A) + l1(rec_B, real_B)) / 2
    loss_grad_cycle = (gradient_loss(rec_A, real_A) + gradient_loss(rec_B, real_B)) / 2
    loss_grad_id = (gradient_loss(id_A, real_A) + gradient_loss(id_B, real_B)) / 2
    loss_ssim = 1 - (ssim(rec_A, real_A) + ssim(rec_B, real_B)) / 2
    loss_ca = contrast_attention_loss(fake_B, real_B, real_A, 0.15, 1.0, 3.0, 7)
    loss_cr = contrast_region_loss(fake_B, real_B, real_A, 0.15, 1.5)
    loss_ce = contrast_edge_loss(fake_B, real_B, real_A)
    loss_G = (loss_GAN + lambda_cyc * loss_cycle + lambda_id * loss_id
              + LAMBDA_GRAD * loss_grad_cycle + LAMBDA_GRAD_ID * loss_grad_id
              + LAMBDA_SSIM * loss_ssim + LAMBDA_CA * loss_ca + LAMBDA_CR * loss_cr
              + LAMBDA_CE * loss_ce)
    return {"loss_G": loss_G, "loss_GAN": loss_GAN, "loss_cycle": loss_cycle, "loss_id": loss_id,
            "loss_grad_cycle": loss_grad_cycle, "loss_grad_id": loss_grad_id, "loss_ssim": loss_ssim,
            "loss_contrast_attention": loss_ca, "loss_contrast_region": loss_cr,
            "loss_contrast_edge": loss_ce}


class OracleCycleGAN:
    """Four parameter dicts + three torch.optim.Adam, exactly as trainer.py:327-367 builds them."""

    def __init__(self, sd_gab: Params, sd_gba: Params, sd_da: Params, sd_db: Params,
                 num_residual_blocks: int, lr: float = 2e-4, lambda_cyc: float = 10.0,
                 lambda_id: float = 5.0, use_cbam: bool = True):
        mk = lambda sd: {k: v.detach().clone().float().requires_grad_(True) for k, v in sd.items()}
        self.G_AB, self.G_BA, self.D_A, self.D_B = mk(sd_gab), mk(sd_gba), mk(sd_da), mk(sd_db)
        self.nb = num_residual_blocks
        self.use_cbam = use_cbam
        self.lambda_cyc, self.lambda_id = lambda_cyc, lambda_id
        betas = (0.5, 0.999)
        self.opt_G = torch.optim.Adam(list(self.G_AB.values()) + list(self.G_BA.values()),
                                      lr=lr, betas=betas)
        self.opt_DA = torch.optim.Adam(list(self.D_A.values()), lr=lr, betas=betas)
        self.opt_DB = torch.optim.Adam(list(self.D_B.values()), lr=lr, betas=betas)

    def G(self, p, x):
        return generator_forward(p, x, self.nb, self.use_cbam)

    def step(self, real_A, real_B, masks=None) -> Dict[str, float]:
        """One pass of modules/trainer.py:447-525 (G step, D_A step, D_B step)."""
        cat = (lambda t: torch.cat([t, masks], 1)) if masks is not None else (lambda t: t)
        rA_in, rB_in = cat(real_A), cat(real_B)
        n, _, H, W = real_A.shape
        valid = torch.ones(n, 1, H // 16, W // 16)
        fake = torch.zeros(n, 1, H // 16, W // 16)

        self.opt_G.zero_grad()
        fake_B, fake_A = self.G(self.G_AB, rA_in), self.G(self.G_BA, rB_in)
        id_A, id_B = self.G(self.G_BA, rA_in), self.G(self.G_AB, rB_in)
        loss_GAN = (mse(discriminator_forward(self.D_B, fake_B), valid)
                    + mse(discriminator_forward(self.D_A, fake_A), valid)) / 2
        rec_A, rec_B = self.G(self.G_BA, cat(fake_B)), self.G(self.G_AB, cat(fake_A))
        T = g_loss_terms(real_A, real_B, rec_A, rec_B, id_A, id_B, fake_B, None, None,
                         self.lambda_cyc, self.lambda_id, loss_GAN=loss_GAN)
        loss_G = T["loss_G"]
        loss_G.backward()
        self.opt_G.step()

        self.opt_DA.zero_grad()
        loss_D_A = (mse(discriminator_forward(self.D_A, real_A), valid)
                    + mse(discriminator_forward(self.D_A, fake_A.detach()), fake)) / 2
        loss_D_A.backward()
        self.opt_DA.step()
        self.opt_DB.zero_grad()
        loss_D_B = (mse(discriminator_forward(self.D_B, real_B), valid)
                    + mse(discriminator_forward(self.D_B, fake_B.detach()), fake)) / 2
        loss_D_B.backward()
        self.opt_DB.step()
        out = {k: float(v.detach()) for k, v in T.items()}
        out.update(loss_D_A=float(loss_D_A.detach()), loss_D_B=float(loss_D_B.detach()))
        return out


def lr_lambda(epoch: int, epochs: int, decay_epoch: int) -> float:
    """modules/trainer.py:364 LambdaLR factor."""
    return 1.0 - max(0, epoch + 1 - decay_epoch) / (epochs - decay_epoch)
