"""Op-level parity of the HIP kernels against fp32 torch-CPU references of the same op.

Every test here is @pytest.mark.gpu and calls the kernels through the C-ABI (ctypes).
Tolerances: fp32 everywhere; max abs error / max |ref| <= 1e-4 for single ops (1e-3 rel for
chained backward passes), following BASELINE.json's 1e-3 rel bar.
"""
import os
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import prng
from oracle import ref_torch as orc

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / max(b.abs().max(), 1e-12))


def rnd(shape, seed, name, lo=-1.0, hi=1.0):
    return torch.from_numpy(prng.uniform(seed, name, shape, lo, hi))


@pytest.fixture(scope="module")
def ops():
    from modules.hip import ops as o
    return o


def torch_conv(x_nchw, w, geom, bias=None):
    """CPU reference of ConvGeom.forward: pad module (+upsample) + F.conv2d."""
    from modules.hip.lib import DCS_PAD_REFLECT
    x = x_nchw
    if geom.up == 2:
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    t, l, b, r = geom.pads
    x = F.pad(x, (l, r, t, b), mode="reflect" if geom.pad_mode == DCS_PAD_REFLECT else "constant")
    return F.conv2d(x, w, bias, stride=geom.stride)


CONV_CASES = [
    # cin, cout, k, stride, pads, mode, up, H
    (3, 64, 7, 1, (3, 3, 3, 3), "reflect", 1, 20),      # stem (scalar gather, cin 3)
    (64, 128, 3, 2, (1, 1, 1, 1), "zero", 1, 18),       # down1
    (128, 256, 3, 2, (1, 1, 1, 1), "zero", 1, 10),      # down2
    (256, 256, 3, 1, (1, 1, 1, 1), "reflect", 1, 9),    # residual
    (256, 128, 3, 1, (1, 1, 1, 1), "zero", 2, 5),       # up1
    (128, 64, 3, 1, (1, 1, 1, 1), "zero", 2, 6),        # up2
    (64, 1, 7, 1, (3, 3, 3, 3), "reflect", 1, 12),      # head (narrow)
    (32, 1, 3, 1, (1, 1, 1, 1), "zero", 1, 10),         # 'same' 3x3 onto one channel (dcs_conv_dgrad_c1)
    (1, 64, 4, 2, (1, 1, 1, 1), "zero", 1, 32),         # D layer 0 (cin 1)
    (64, 128, 4, 2, (1, 1, 1, 1), "zero", 1, 16),       # D layer 1
    (256, 512, 4, 2, (1, 1, 1, 1), "zero", 1, 8),       # D layer 3
    (512, 1, 4, 1, (2, 2, 1, 1), "zero", 1, 4),         # D last (narrow, asymmetric pad)
    (256, 1, 4, 1, (2, 2, 1, 1), "zero", 1, 9),         # one-wave-per-pixel kernel, 4 channels per lane
    # the layer shapes of a 64x64 generator at batch 1 (split-K wgrad, multi-tile rows)
    (256, 128, 3, 1, (1, 1, 1, 1), "zero", 2, 16),
    (128, 64, 3, 1, (1, 1, 1, 1), "zero", 2, 32),
    (64, 1, 7, 1, (3, 3, 3, 3), "reflect", 1, 64),
    (256, 256, 3, 1, (1, 1, 1, 1), "reflect", 1, 16),
    (64, 128, 3, 2, (1, 1, 1, 1), "zero", 1, 64),
]


def _geom(case):
    from modules.hip.ops import ConvGeom
    from modules.hip.lib import DCS_PAD_REFLECT, DCS_PAD_ZERO
    cin, cout, k, s, pads, mode, up, H = case
    return ConvGeom(cin, cout, k, s, pads, DCS_PAD_REFLECT if mode == "reflect" else DCS_PAD_ZERO, up), H


@pytest.mark.parametrize("case", CONV_CASES, ids=[f"c{c[0]}-{c[1]}k{c[2]}s{c[3]}u{c[6]}" for c in CONV_CASES])
def test_conv_fwd_dgrad_wgrad(ops, case):
    torch.manual_seed(0)
    g, H = _geom(case)
    N = 2 if H < 16 else 1
    x = rnd((N, g.cin, H, H + 1), 1, "x")
    w = torch.from_numpy(prng.normal(2, "w", (g.cout, g.cin, g.k, g.k), 0, 0.05))
    bias = rnd((g.cout,), 3, "b")
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = torch_conv(xr, wr, g, bias)
    R = torch.from_numpy(prng.normal(4, "R", tuple(yr.shape)))
    (yr * R).sum().backward()

    xd = x.to(DEV).permute(0, 2, 3, 1).contiguous()
    wd, bd = w.to(DEV), bias.to(DEV)
    y = g.forward(ops.Src.nhwc(xd), g.pack_fwd(wd), bias=bd)
    assert rel(y.permute(0, 3, 1, 2), yr) < 1e-4
    Rd = R.to(DEV).permute(0, 2, 3, 1).contiguous()
    dw = g.wgrad(Rd, ops.Src.nhwc(xd))
    assert rel(dw, wr.grad) < 1e-4
    dx = g.dgrad(Rd, g.pack_dgrad(wd), H, H + 1)
    assert rel(dx.permute(0, 3, 1, 2), xr.grad) < 1e-4


def test_conv_prologue_and_concat(ops):
    """IN+ReLU prologue and channel-concat of two NCHW sources fused in the gather."""
    from modules.hip.ops import ConvGeom, Src
    from modules.hip.lib import ACT_RELU, DCS_PAD_REFLECT
    N, H, W = 2, 16, 12
    img = rnd((N, 1, H, W), 5, "img")
    masks = (rnd((N, 2, H, W), 6, "m", 0, 1) < 0.3).float()
    g = ConvGeom(3, 64, 7, 1, (3, 3, 3, 3), DCS_PAD_REFLECT)
    w = torch.from_numpy(prng.normal(7, "w", (64, 3, 7, 7), 0, 0.05))
    ref = torch_conv(torch.cat([img, masks], 1), w, g)
    y = g.forward(Src.nchw(img.to(DEV), masks.to(DEV)), g.pack_fwd(w.to(DEV)))
    assert rel(y.permute(0, 3, 1, 2), ref) < 1e-4
    # prologue: next conv consumes relu(IN(y))
    st = ops.in_stats(y)
    g2 = ConvGeom(64, 128, 3, 2, (1, 1, 1, 1))
    w2 = torch.from_numpy(prng.normal(8, "w2", (128, 64, 3, 3), 0, 0.05))
    a = F.relu(F.instance_norm(ref, eps=1e-5))
    ref2 = torch_conv(a, w2, g2)
    y2 = g2.forward(Src.nhwc(y), g2.pack_fwd(w2.to(DEV)), pro=(st.scale, st.shift, ACT_RELU))
    assert rel(y2.permute(0, 3, 1, 2), ref2) < 1e-4


@pytest.mark.parametrize("N,C,H,W", [(3, 64, 17, 13), (3, 256, 8, 8), (3, 512, 4, 4), (3, 128, 32, 32),
                                     (1, 128, 32, 32), (1, 64, 64, 64), (2, 256, 64, 64)])
def test_instance_norm(ops, N, C, H, W):
    from modules.hip.lib import ACT_LRELU, ACT_RELU
    x = rnd((N, C, H, W), 9, "x", -2, 3)
    xd = x.to(DEV).permute(0, 2, 3, 1).contiguous()
    st = ops.in_stats(xd, want_max=True)
    ref = F.instance_norm(x, eps=1e-5)
    for act, fn in ((ACT_RELU, F.relu), (ACT_LRELU, lambda t: F.leaky_relu(t, 0.2))):
        out = ops.in_apply(xd, st, act)
        assert rel(out.permute(0, 3, 1, 2), fn(ref)) < 1e-5
        xr = x.clone().requires_grad_(True)
        yr = fn(F.instance_norm(xr, eps=1e-5))
        R = torch.from_numpy(prng.normal(10, "R", tuple(yr.shape)))
        (yr * R).sum().backward()
        dy = ops.in_act_backward(R.to(DEV).permute(0, 2, 3, 1).contiguous(), xd, st, act)
        assert rel(dy.permute(0, 3, 1, 2), xr.grad) < 1e-4
    mx, am = x.flatten(2).max(-1)
    assert torch.equal(st.xmax.cpu(), mx)
    assert torch.equal(st.xargmax.cpu().long(), am)


def test_cbam_tail(ops):
    """out = x + CBAM(IN(y)) forward and backward (incl. IN backward) vs the oracle."""
    N, C, H, W = 2, 256, 12, 10
    x = torch.from_numpy(prng.normal(11, "x", (N, C, H, W)))
    y = torch.from_numpy(prng.normal(12, "y", (N, C, H, W), 0.3, 1.7))
    w1 = torch.from_numpy(prng.normal(13, "w1", (16, C, 1, 1), 0, 0.1))
    w2 = torch.from_numpy(prng.normal(14, "w2", (C, 16, 1, 1), 0, 0.1))
    wsa = torch.from_numpy(prng.normal(15, "wsa", (1, 2, 7, 7), 0, 0.1))
    P = {"c.channel_attention.fc.0.weight": w1.clone().requires_grad_(True),
         "c.channel_attention.fc.2.weight": w2.clone().requires_grad_(True),
         "c.spatial_attention.conv.weight": wsa.clone().requires_grad_(True)}
    xr, yr = x.clone().requires_grad_(True), y.clone().requires_grad_(True)
    z = F.instance_norm(yr, eps=1e-5)
    z = orc.channel_attention(P, "c.channel_attention", z)
    z = orc.spatial_attention(P, "c.spatial_attention", z)
    outr = xr + z
    R = torch.from_numpy(prng.normal(16, "R", tuple(outr.shape)))
    (outr * R).sum().backward()

    xd = x.to(DEV).permute(0, 2, 3, 1).contiguous()
    yd = y.to(DEV).permute(0, 2, 3, 1).contiguous()
    st = ops.in_stats(yd, want_max=True)
    w1d, w2d, wsad = w1.to(DEV).view(16, C), w2.to(DEV).view(C, 16), wsa.to(DEV).view(2, 7, 7)
    out, saved = ops.cbam_forward(xd, yd, st, w1d, w2d, wsad)
    assert rel(out.permute(0, 3, 1, 2), outr) < 1e-4
    dy, dw1, dw2, dwsa = ops.cbam_backward(R.to(DEV).permute(0, 2, 3, 1).contiguous(), yd, st, w1d,
                                           w2d, wsad, saved)
    assert rel(dy.permute(0, 3, 1, 2), yr.grad) < 1e-3
    assert rel(dw1.view_as(w1), P["c.channel_attention.fc.0.weight"].grad) < 1e-3
    assert rel(dw2.view_as(w2), P["c.channel_attention.fc.2.weight"].grad) < 1e-3
    assert rel(dwsa.view_as(wsa), P["c.spatial_attention.conv.weight"].grad) < 1e-3


LOSS_CASES = {
    "l1": (lambda o, p, t, s: o.loss_l1(p, t), lambda p, t, s: orc.l1(p, t)),
    "mse": (lambda o, p, t, s: o.loss_mse(p, t), lambda p, t, s: orc.mse(p, t)),
    "mse_const": (lambda o, p, t, s: o.loss_mse_const(p, 1.0), lambda p, t, s: orc.mse(p, torch.ones_like(p))),
    "gradient": (lambda o, p, t, s: o.loss_gradient(p, t), lambda p, t, s: orc.gradient_loss(p, t)),
    "contrast_attention": (lambda o, p, t, s: o.loss_contrast_attention(p, t, s, 0.15, 1.0, 3.0, 7),
                           lambda p, t, s: orc.contrast_attention_loss(p, t, s, 0.15, 1.0, 3.0, 7)),
    "contrast_region": (lambda o, p, t, s: o.loss_contrast_region(p, t, s, 0.15, 1.5),
                        lambda p, t, s: orc.contrast_region_loss(p, t, s, 0.15, 1.5)),
    "contrast_edge": (lambda o, p, t, s: o.loss_contrast_edge(p, t),
                      lambda p, t, s: orc.contrast_edge_loss(p, t, s)),
    "ssim": (lambda o, p, t, s: o.loss_ssim(p, t, 1.0), lambda p, t, s: orc.ssim(p, t, 1.0)),
}


@pytest.mark.parametrize("shape", [(2, 1, 64, 64), (1, 1, 48, 40), (3, 1, 33, 47)])
@pytest.mark.parametrize("name", sorted(LOSS_CASES))
def test_losses(ops, name, shape):
    hip_fn, ref_fn = LOSS_CASES[name]
    p = torch.tanh(torch.from_numpy(prng.normal(17, "p", shape)))
    t = rnd(shape, 18, "t")
    s = rnd(shape, 19, "s")
    pr = p.clone().requires_grad_(True)
    vr = ref_fn(pr, t, s)
    vr.backward()
    v, g = hip_fn(ops, p.to(DEV), t.to(DEV), s.to(DEV))
    assert abs(float(v) - float(vr)) <= 1e-5 * max(1.0, abs(float(vr))), (name, float(v), float(vr))
    assert rel(g, pr.grad) < 1e-4, name


def test_adam_matches_torch(ops):
    n = 10000
    p0 = torch.from_numpy(prng.normal(20, "p", (n,)))
    opt_p = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([opt_p], lr=2e-4, betas=(0.5, 0.999))
    pd, md, vd = p0.to(DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    for step in range(1, 4):
        g = torch.from_numpy(prng.normal(21, f"g{step}", (n,)))
        opt_p.grad = g.clone()
        opt.step()
        ops.adam_step(pd, g.to(DEV), md, vd, 2e-4, 0.5, 0.999, 1e-8, step)
    assert rel(pd, opt_p.detach()) < 1e-6


def test_integration_md_ctypes_example(ops):
    """The stand-alone ctypes snippet in INTEGRATION.md runs as written (from the repo root) and
    matches torch's reflect-padded conv on the CPU."""
    import re
    import torch.nn.functional as F
    from conftest import ROOT
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    code = re.search(r"```python\n(.*?)```", text, re.S).group(1)
    code = code.replace("N, H, W, C = 8, 128, 128, 256", "N, H, W, C = 2, 16, 16, 256")
    code = code.replace('"ducosy-gan_amd/lib/libducosy_hip.so"', repr(os.path.join(ROOT, "ducosy-gan_amd", "lib",
                                                                                 "libducosy_hip.so")))
    env = {}
    exec(compile(code, "INTEGRATION.md", "exec"), env)
    torch.cuda.synchronize()
    x, w, y = env["x"].cpu(), env["w"].cpu(), env["y"].cpu()
    ref = F.conv2d(F.pad(x.permute(0, 3, 1, 2), (1, 1, 1, 1), mode="reflect"), w).permute(0, 2, 3, 1)
    assert float((y - ref).abs().max()) <= 1e-4 * float(ref.abs().max())


@pytest.mark.parametrize("H", [3, 4, 9, 16])
def test_reflect_dgrad_direct_and_accumulate(ops, H):
    """Residual-conv data gradient (padded-grid transposed conv + reflection fold) against
    autograd through F.pad(reflect) + conv2d, with and without the residual addend, down to
    the smallest reflectable size."""
    g, _ = _geom((256, 256, 3, 1, (1, 1, 1, 1), "reflect", 1, H))
    x = rnd((2, 256, H, H), 31, "x").requires_grad_(True)
    w = rnd((256, 256, 3, 3), 31, "w", -0.05, 0.05)
    dy = rnd((2, 256, H, H), 31, "dy")
    torch_conv(x, w, g).backward(dy)
    wd = g.pack_dgrad(w.cuda())
    dyn = dy.permute(0, 2, 3, 1).contiguous().cuda()
    dx = g.dgrad(dyn, wd, H, H)
    assert rel(dx.permute(0, 3, 1, 2), x.grad) < 1e-4
    add = rnd((2, H, H, 256), 31, "add").cuda()
    want = dx + add
    got = g.dgrad(dyn, wd, H, H, addend=add.clone())
    assert rel(got, want) < 1e-5


@pytest.mark.parametrize("H,mode", [(4, "bf16x6"), (9, "bf16x6"), (16, "f32"), (16, "bf16x6"), (9, "f16x3"), (16, "f16x3")])
def test_dgrad_reflect_epilogue_fold_matches_fold_pass(ops, H, mode):
    """dcs_conv_dgrad_reflect (interior pixels stored by the conv epilogue, the one-pixel ring
    folded in by a second kernel) against the padded-grid pass + dcs_reflect_fold, without and
    (direct C-ABI call) with the residual addend; only the summation order of the ring pixels
    differs."""
    import ctypes
    from modules.hip import lib
    prev = ops.get_mma()
    ops.set_mma(mode)
    try:
        g, _ = _geom((256, 256, 3, 1, (1, 1, 1, 1), "reflect", 1, H))
        w = rnd((256, 256, 3, 3), 41, "w", -0.05, 0.05).cuda()
        wd = g.pack_dgrad(w)
        dyn = rnd((2, H, H, 256), 41, "dy").cuda()
        add = rnd((2, H, H, 256), 41, "add").cuda()
        fused = g.dgrad(dyn, wd, H, H)  # f16x3 at H = 16: the window pass (csrc/conv_win.hip)
        ops._FUSE_FOLD, ops._WIN = False, False
        try:
            plain = g.dgrad(dyn, wd, H, H)
            plain_add = g.dgrad(dyn, wd, H, H, addend=add.clone())
        finally:
            ops._FUSE_FOLD, ops._WIN = True, True
        # the window pass sums in another order (one chain per 16-channel slice)
        assert rel(fused, plain) < (2e-6 if g.win else 1e-6)
        d = lib.ConvDesc()
        d.N, d.Hs, d.Ws, d.Cs = 2, H, H, 256
        d.s_n, d.s_c, d.s_h, d.s_w = H * H * 256, 1, H * 256, 256
        d.csplit, d.up, d.pad_mode = 256, 1, lib.DCS_PAD_ZERO
        d.KH = d.KW = 3
        d.pt = d.pl = 2
        d.stride, d.Ho, d.Wo, d.Co = 1, H + 2, H + 2, 256
        d.ldb = wd.shape[1]
        ops._set_mma(d, dyn, None, ops._wrng(wd))  # f16x3: the operands' range records
        d.korder = lib.KORDER_SLICE if g.kslice else lib.KORDER_TAP
        ring = lib.query("dcs_conv_dgrad_reflect_ring_size", ctypes.byref(d)) // 4
        buf = torch.empty(2 * H * H * 256 + ring, device=DEV)
        lib.call("dcs_conv_dgrad_reflect", ctypes.byref(d), ctypes.c_void_p(dyn.data_ptr()),
                 ctypes.c_void_p(wd.data_ptr()), ctypes.c_void_p(add.data_ptr()), ctypes.c_void_p(buf.data_ptr()),
                 ctypes.c_void_p(buf.data_ptr() + 2 * H * H * 256 * 4), None)
        torch.cuda.synchronize()
        assert rel(buf[:2 * H * H * 256].view(2, H, H, 256), plain_add) < 1e-6
    finally:
        ops.set_mma(prev)


@pytest.mark.parametrize("c1,c2,k,stride,pads,mode", [(1, 2, 7, 1, (3, 3, 3, 3), "reflect"),
                                                      (1, 1, 7, 1, (3, 3, 3, 3), "reflect"),
                                                      (1, 0, 7, 1, (3, 3, 3, 3), "reflect"),
                                                      (1, 0, 4, 2, (1, 1, 1, 1), "zero")])
def test_four_channel_stem_path(ops, c1, c2, k, stride, pads, mode):
    """Image (+ mask planes) packed NHWC x 4 (dcs_pack_nhwc4) and the float4-per-tap gather
    (stem 7x7 and PatchGAN layer 0): forward and weight gradient vs torch on the concat, and the
    data gradient onto the image channel (dcs_conv_dgrad_to1; odd width)."""
    from modules.hip.ops import ConvGeom, Src
    from modules.hip.lib import DCS_PAD_REFLECT, DCS_PAD_ZERO
    cin, H, W = c1 + c2, 36, 37
    g = ConvGeom(cin, 64, k, stride, pads, DCS_PAD_REFLECT if mode == "reflect" else DCS_PAD_ZERO)
    x = rnd((2, c1, H, W), 41, "x").requires_grad_(True)
    m = rnd((2, c2, H, W), 41, "m") if c2 else None
    w = rnd((64, cin, k, k), 41, "w", -0.1, 0.1).requires_grad_(True)
    xc = torch.cat([x, m], 1) if c2 else x
    y_ref = torch_conv(xc, w, g)
    dy = rnd(tuple(y_ref.shape), 41, "dy")
    y_ref.backward(dy)
    xd = x.detach().cuda()
    x4 = ops.pack_nhwc4(xd, m.cuda() if c2 else None)
    assert x4.shape == (2, H, W, 4)
    assert torch.equal(x4[..., :cin].cpu(), xc.detach().permute(0, 2, 3, 1))
    assert float(x4[..., cin:].abs().max()) == 0.0 if cin < 4 else True
    s4 = Src.nhwc(x4)
    y = g.forward(s4, g.pack_fwd(w.detach().cuda(), cin_pad=4))
    assert rel(y.permute(0, 3, 1, 2), y_ref) < 1e-4
    dyn = dy.permute(0, 2, 3, 1).contiguous().cuda()
    dw = g.wgrad(dyn, s4)
    assert dw.shape == w.shape
    assert rel(dw, w.grad) < 1e-4
    assert g.to1_dgrad(1)
    dx = g.dgrad(dyn, g.pack_dgrad(w.detach().cuda(), 1), H, W, ci_count=1)
    assert dx.shape == (2, H, W, 1)
    assert rel(dx.permute(0, 3, 1, 2), x.grad) < 1e-5
    add = rnd((2, H, W, 1), 42, "add").cuda()
    got = g.dgrad(dyn, g.pack_dgrad(w.detach().cuda(), 1), H, W, ci_count=1, addend=add)
    assert rel(got, dx + add) < 1e-6


STATS_CASES = [
    # cin, cout, k, stride, pads, mode, up, N, H, W, pro, want_max
    (256, 256, 3, 1, (1, 1, 1, 1), "reflect", 1, 2, 16, 16, False, True),   # residual (256-row x6 tiles)
    (256, 256, 3, 1, (1, 1, 1, 1), "reflect", 1, 3, 16, 24, False, True),   # residual, 384 rows (128-row tiles)
    (64, 128, 3, 2, (1, 1, 1, 1), "zero", 1, 2, 32, 32, False, False),      # down1
    (256, 128, 3, 1, (1, 1, 1, 1), "zero", 2, 2, 16, 16, False, False),     # up1 (sub-pixel phases)
    (64, 128, 4, 2, (1, 1, 1, 1), "zero", 1, 2, 32, 32, True, False),       # PatchGAN layer 1 (LReLU prologue)
]


@pytest.mark.parametrize("mode", ["f32", "bf16x6", "f16x3"])
@pytest.mark.parametrize("case", STATS_CASES, ids=[f"c{c[0]}-{c[1]}k{c[2]}s{c[3]}u{c[6]}N{c[7]}H{c[8]}W{c[9]}"
                                                   for c in STATS_CASES])
def test_forward_in_stats_matches_stats_pass(ops, mode, case):
    """IN statistics from the conv epilogue (dcs_conv_rows_in_stats + dcs_in_stats_finish) ==
    forward + the statistics pass: the same output bits, scale / shift to fp32 rounding, the same
    max and first argmax."""
    from modules.hip.lib import ACT_LRELU, DCS_PAD_REFLECT, DCS_PAD_ZERO
    from modules.hip.ops import ConvGeom, Src
    cin, cout, k, s, pads, pm, up, N, H, W, pro, want_max = case
    g = ConvGeom(cin, cout, k, s, pads, DCS_PAD_REFLECT if pm == "reflect" else DCS_PAD_ZERO, up)
    prev = ops.get_mma()
    ops.set_mma(mode)
    try:
        x = rnd((N, H, W, cin), 51, f"sx{cin}{H}{W}").cuda()
        w = torch.from_numpy(prng.normal(52, f"sw{cin}{cout}", (cout, cin, k, k), 0, 0.05)).cuda()
        p = None
        if pro:
            st0 = ops.in_stats(x)
            p = (st0.scale, st0.shift, ACT_LRELU)
        wp = g.pack_fwd(w)
        y_ref = g.forward(Src.nhwc(x), wp, pro=p)
        s_ref = ops.in_stats(y_ref, want_max=want_max)
        y, st = g.forward_in_stats(Src.nhwc(x), wp, pro=p, want_max=want_max)
        torch.cuda.synchronize()
    finally:
        ops.set_mma(prev)
    assert torch.equal(y, y_ref)
    assert rel(st.scale, s_ref.scale) < 2e-6
    assert float((st.shift - s_ref.shift).abs().max()) < 2e-6 * max(1.0, float(s_ref.shift.abs().max()))
    if want_max:
        assert torch.equal(st.xmax, s_ref.xmax)
        assert torch.equal(st.xargmax, s_ref.xargmax)
    # and the fused path really ran (rows per image % 128 == 0 here)
    import ctypes
    from modules.hip import lib
    d = g._desc_fwd(Src.nhwc(x), wp.shape[1], p[2] if p else 0, 0)
    assert lib.query("dcs_conv_rows_in_stats_parts_size", ctypes.byref(d)) > 0


@pytest.mark.parametrize("P,C", [(1, 1), (1000, 1), (512 * 512 * 2 + 3, 1), (4097, 3), (33 * 33, 64),
                                 (256 * 256, 64), (70, 256), (5000, 512)])
def test_channel_sum(ops, P, C):
    """Bias gradients (sum over pixels per channel), both the flat power-of-two pass and the
    per-channel one, against a float64 sum; ragged tails included."""
    x = rnd((P, C), 17, f"cs{P}_{C}").to(DEV)
    got = ops.channel_sum(x)
    ref = x.double().sum(0)
    assert float((got.double() - ref).abs().max()) <= 1e-5 * max(1.0, float(x.abs().sum(0).max()))
