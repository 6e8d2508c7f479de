"""Drop-in mirror of the reference's modules/model.py on the MI355X kernel library.

Same class names, constructor signatures, nn.Sequential indices, state_dict keys/shapes and
.parameters() order as modules/model.py:6-140, so reference checkpoints load unchanged and
optimizer state lines up.  The module tree is the parameter skeleton; ``Generator.forward``,
``Discriminator.forward`` and ``ResidualBlock[WithCBAM].forward`` run the fused HIP path
(modules/hip/networks.py) and require device tensors — there is no CPU fallback.

``ChannelAttention`` / ``SpatialAttention`` / ``CBAM`` keep a standalone torch forward for API
completeness only; inside the residual blocks (the hot path) CBAM runs as fused HIP kernels.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .hip import networks as _net


# ---- CBAM (Convolutional Block Attention Module) — modules/model.py:6-52 ----
class ChannelAttention(nn.Module):
    """modules/model.py:6-24 (standalone forward is a convenience, not the hot path)."""

    def __init__(self, channels, reduction=16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.max_pool = nn.AdaptiveMaxPool2d(1)
        self.fc = nn.Sequential(nn.Conv2d(channels, channels // reduction, 1, bias=False),
                                nn.ReLU(inplace=True),
                                nn.Conv2d(channels // reduction, channels, 1, bias=False))
        self.sigmoid = nn.Sigmoid()

    def forward(self, x):
        return x * self.sigmoid(self.fc(self.avg_pool(x)) + self.fc(self.max_pool(x)))


class SpatialAttention(nn.Module):
    """modules/model.py:27-39 (standalone forward is a convenience, not the hot path)."""

    def __init__(self, kernel_size=7):
        super().__init__()
        self.conv = nn.Conv2d(2, 1, kernel_size, padding=kernel_size // 2, bias=False)
        self.sigmoid = nn.Sigmoid()

    def forward(self, x):
        s = torch.cat([x.mean(dim=1, keepdim=True), x.max(dim=1, keepdim=True)[0]], dim=1)
        return x * self.sigmoid(self.conv(s))


class CBAM(nn.Module):
    """modules/model.py:42-52."""

    def __init__(self, channels, reduction=16, kernel_size=7):
        super().__init__()
        self.channel_attention = ChannelAttention(channels, reduction)
        self.spatial_attention = SpatialAttention(kernel_size)

    def forward(self, x):
        return self.spatial_attention(self.channel_attention(x))


# ---- residual blocks — modules/model.py:56-87 ----
def _block_params(blk, use_cbam):
    keys = ["r0.c1.w", "r0.c1.b", "r0.c2.w", "r0.c2.b"]
    params = [blk.block[1].weight, blk.block[1].bias, blk.block[5].weight, blk.block[5].bias]
    if use_cbam:
        keys += ["r0.fc1", "r0.fc2", "r0.sa"]
        params += [blk.cbam.channel_attention.fc[0].weight, blk.cbam.channel_attention.fc[2].weight,
                   blk.cbam.spatial_attention.conv.weight]
    return keys, params


class ResidualBlock(nn.Module):
    """x + [ReflPad, Conv3x3, IN, ReLU, ReflPad, Conv3x3, IN](x)  (modules/model.py:56-65)."""

    def __init__(self, in_features):
        super().__init__()
        self.block = nn.Sequential(
            nn.ReflectionPad2d(1), nn.Conv2d(in_features, in_features, 3), nn.InstanceNorm2d(in_features),
            nn.ReLU(inplace=True), nn.ReflectionPad2d(1), nn.Conv2d(in_features, in_features, 3),
            nn.InstanceNorm2d(in_features))

    def forward(self, x):
        keys, params = _block_params(self, False)
        return _net.ResBlockFunction.apply(x, False, tuple(keys), *params)


class ResidualBlockWithCBAM(nn.Module):
    """x + CBAM(block(x))  (modules/model.py:68-87)."""

    def __init__(self, in_features):
        super().__init__()
        self.block = nn.Sequential(
            nn.ReflectionPad2d(1), nn.Conv2d(in_features, in_features, 3), nn.InstanceNorm2d(in_features),
            nn.ReLU(inplace=True), nn.ReflectionPad2d(1), nn.Conv2d(in_features, in_features, 3),
            nn.InstanceNorm2d(in_features))
        self.cbam = CBAM(in_features)

    def forward(self, x):
        keys, params = _block_params(self, True)
        return _net.ResBlockFunction.apply(x, True, tuple(keys), *params)


# ---- networks — modules/model.py:90-131 ----
class Generator(nn.Module):
    """ResNet generator with CBAM (modules/model.py:90-115); output 1 channel, tanh."""

    def __init__(self, input_channels=1, num_residual_blocks=9, use_cbam=True):
        super().__init__()
        model = [nn.ReflectionPad2d(3), nn.Conv2d(input_channels, 64, 7), nn.InstanceNorm2d(64),
                 nn.ReLU(inplace=True)]
        in_features, out_features = 64, 128
        for _ in range(2):
            model += [nn.Conv2d(in_features, out_features, 3, stride=2, padding=1),
                      nn.InstanceNorm2d(out_features), nn.ReLU(inplace=True)]
            in_features, out_features = out_features, out_features * 2
        for _ in range(num_residual_blocks):
            model += [ResidualBlockWithCBAM(in_features) if use_cbam else ResidualBlock(in_features)]
        out_features = in_features // 2
        for _ in range(2):
            model += [nn.Upsample(scale_factor=2), nn.Conv2d(in_features, out_features, 3, stride=1, padding=1),
                      nn.InstanceNorm2d(out_features), nn.ReLU(inplace=True)]
            in_features, out_features = out_features, out_features // 2
        model += [nn.ReflectionPad2d(3), nn.Conv2d(in_features, 1, 7), nn.Tanh()]
        self.model = nn.Sequential(*model)
        self.input_channels = input_channels
        self.num_residual_blocks = num_residual_blocks
        self.use_cbam = use_cbam
        inv = {v: k for k, v in _net.gen_param_names(num_residual_blocks, use_cbam).items()}
        self._keys = tuple(inv[name] for name, _ in self.named_parameters())

    def forward(self, x, masks=None, input_grad_from=0):
        """x: [N, input_channels, H, W] (the reference's concat input) — or the image channels
        with ``masks`` given separately, in which case the concat is fused into the stem.
        ``input_grad_from``: the samples before this index are data whose input gradient nobody
        reads (a batch concatenated from real images and one generated tensor); the input
        gradient is computed for x[input_grad_from:] only and is zero before it."""
        params = [p for _, p in self.named_parameters()]
        cfg = (self._keys, self.num_residual_blocks, self.use_cbam, int(input_grad_from))
        return _net.GeneratorFunction.apply(x, masks, cfg, *params)


class Discriminator(nn.Module):
    """70x70 PatchGAN (modules/model.py:118-131)."""

    def __init__(self, input_channels=1):
        super().__init__()

        def block(in_f, out_f, norm=True):
            layers = [nn.Conv2d(in_f, out_f, 4, stride=2, padding=1)]
            if norm:
                layers.append(nn.InstanceNorm2d(out_f))
            layers.append(nn.LeakyReLU(0.2, inplace=True))
            return layers

        self.model = nn.Sequential(
            *block(input_channels, 64, norm=False), *block(64, 128), *block(128, 256), *block(256, 512),
            nn.ZeroPad2d((1, 0, 1, 0)), nn.Conv2d(512, 1, 4, padding=1))

    def forward(self, img, params_require_grad=True):
        params = [p for _, p in self.named_parameters()]
        if not params_require_grad:  # G step: gradient w.r.t. the input only (trainer.py:470)
            params = [p.detach() for p in params]
        return _net.DiscriminatorFunction.apply(img, *params)


def weights_init_normal(m):
    """modules/model.py:134-140: conv weights ~ N(0, 0.02)."""
    classname = m.__class__.__name__
    if classname.find("Conv") != -1:
        torch.nn.init.normal_(m.weight.data, 0.0, 0.02)
    elif classname.find("BatchNorm2d") != -1:
        torch.nn.init.normal_(m.weight.data, 1.0, 0.02)
        torch.nn.init.constant_(m.bias.data, 0.0)
