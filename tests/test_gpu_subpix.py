"""The sub-pixel window kernel of the Generator's up-convolutions (csrc/conv_subpix.hip;
modules/model.py:112-120: Upsample(x2, nearest) + Conv2d 3x3 pad 1) against float64 references of
the same fp32 operands:
  * forward + the InstanceNorm statistics of its output (scale / shift / max / argmax from the
    epilogue partials) for up1 (256 -> 128) and up2 (128 -> 64) shapes, source widths 16 .. 256
    (every tile width the kernel takes: 16, 32, 64, 128 and two column strips);
  * the fp32-class bound of the rows pass it replaces (max error / max |ref| <= 1e-5) in f16x3 mode;
    in f16 mode every layer runs on fp16 operands since round 6 (ops._PHASE_F16X3 empty; a layer kept
    there takes f16x3 and the 1e-5 bound): 2e-3 against the fp32 operands; the PatchGAN layer (whose
    phase classes split the taps, so its fp16 operands are the taps rounded) also within 1e-4 / 2e-5
    of float64 of the operands rounded to fp16 (the up-convs' phase weights are tap sums rounded once);
  * the data gradient (per phase a 2x2 conv of dy's phase sub-grid with the transposed phase weights)
    against float64 autograd of upsample + conv, to the same bound;
  * the weight gradient (phase weight gradients on a rolling source window, folded onto the 3x3 taps)
    against float64 autograd, to the same bound;
  * the down-convs (stride-2 3x3 zero-pad-1) and the PatchGAN layers (4x4, with the previous layer's
    IN + LeakyReLU staged as a prologue) on the same kernels: forward + statistics over the source's
    parity classes, data gradient over dx's, to the same bound;
  * the weight gradients of those stride-2 layers on the rolling class-window kernel, to the same bound;
  * the data gradients with the IN-backward partial sums fused equal the separate passes;
  * the rows pass on the same pack (the phase planes removed) agrees to its own bound, and the
    batched pack (ops.prepack) equals the per-pack launches bit for bit.
Tolerances written per check below."""
import pytest
import torch
import torch.nn.functional as F

from oracle import prng
from test_gpu_ops import rnd

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _relmax(a, b):
    return float((a.double().cpu() - b).abs().max() / b.abs().max())


@pytest.fixture
def ops():
    from modules.hip import ops as o
    prev = o.get_mma()
    yield o
    o.set_mma(prev)


def _geom(ops, cin, cout):
    from modules.hip.lib import DCS_PAD_ZERO
    return ops.ConvGeom(cin, cout, 3, 1, (1, 1, 1, 1), DCS_PAD_ZERO, up=2)


def _fp16_ops(ops, g, mode):
    """True when the layer's phase kernels take fp16 operands (f16 mode, not in ops._PHASE_F16X3)."""
    return mode == "f16" and g._phase_tag() not in ops._PHASE_F16X3


def _h(t):
    """float64 of t's values rounded to fp16 (the f16 path's operands)."""
    return t.detach().half().double()


@pytest.mark.parametrize("mode", ["f16x3", "f16"])
@pytest.mark.parametrize("cin,cout,N,H,W", [(256, 128, 2, 16, 16), (256, 128, 1, 8, 32), (128, 64, 2, 8, 64),
                                            (128, 64, 1, 4, 128), (128, 64, 1, 2, 256), (96, 64, 1, 8, 32)])
def test_subpix_forward_and_stats_vs_fp64(ops, mode, cin, cout, N, H, W):
    """(cin 96: an odd count of 16-channel slices, the f16 kernel's last barrier with one iteration.)"""
    ops.set_mma(mode)
    g = _geom(ops, cin, cout)
    assert g.subwin
    f16 = _fp16_ops(ops, g, mode)
    tol = 2e-3 if f16 else 1e-5
    x = rnd((N, cin, H, W), 81, "x").double()
    w = torch.from_numpy(prng.normal(82, "w", (cout, cin, 3, 3), 0, 0.05)).float().double()
    ref = F.conv2d(F.interpolate(x, scale_factor=2, mode="nearest"), w, padding=1)
    mean = ref.mean(dim=(2, 3))
    var = ref.var(dim=(2, 3), unbiased=False)
    xd = x.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    wp = g.pack_fwd(w.float().to(DEV))
    assert getattr(wp, "_dcs_sp", None) is not None
    y, st = g.forward_in_stats(ops.Src.nhwc(xd), wp, want_max=True)
    assert _relmax(y.permute(0, 3, 1, 2), ref) <= tol
    rstd = 1.0 / torch.sqrt(var + 1e-5)
    assert _relmax(st.scale, rstd) <= tol
    assert float((st.shift.double().cpu() + mean * rstd).abs().max()) <= tol * float((mean * rstd).abs().max() + 1)
    mx = ref.flatten(2).max(dim=2)
    assert _relmax(st.xmax, mx.values) <= tol
    am = st.xargmax.cpu().long()  # the first maximum; a near-tie within rounding may pick either
    got_at = ref.flatten(2).gather(2, am[..., None])[..., 0]
    assert float((got_at - mx.values).abs().max()) <= tol * float(mx.values.abs().max())
    # forward without statistics: the same values
    y2 = g.forward(ops.Src.nhwc(xd), wp)
    assert torch.equal(y2, y)
    # the rows pass over the same pack (phase planes removed) to the same bound
    sp = wp._dcs_sp
    del wp._dcs_sp
    try:
        y0 = g.forward(ops.Src.nhwc(xd), wp)
    finally:
        wp._dcs_sp = sp
    assert _relmax(y0.permute(0, 3, 1, 2), ref) <= (tol if mode == "f16x3" else 2e-3)  # rows pass: fp16 operands


@pytest.mark.parametrize("mode", ["f16x3", "f16"])
@pytest.mark.parametrize("cin,cout,N,H,W", [(256, 128, 2, 16, 16), (256, 128, 1, 8, 32), (128, 64, 2, 8, 64),
                                            (128, 64, 1, 2, 256)])
def test_subpix_dgrad_vs_fp64(ops, mode, cin, cout, N, H, W):
    """dL/dx of the up-conv (the adjoint of upsample + conv) from dy, against float64 autograd; the rows
    pass over the same pack (phase planes removed) to its own bound."""
    ops.set_mma(mode)
    g = _geom(ops, cin, cout)
    x = rnd((N, cin, H, W), 84, "x").double().requires_grad_(True)
    w = torch.from_numpy(prng.normal(85, "w", (cout, cin, 3, 3), 0, 0.05)).float().double()
    dy = rnd((N, cout, 2 * H, 2 * W), 86, "dy").double()
    y = F.conv2d(F.interpolate(x, scale_factor=2, mode="nearest"), w, padding=1)
    (ref,) = torch.autograd.grad(y, x, dy)
    dyd = dy.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    wd = g.pack_dgrad(w.float().to(DEV))
    assert getattr(wd, "_dcs_sp", None) is not None
    dx = g.dgrad(dyd, wd, H, W)
    assert _relmax(dx.permute(0, 3, 1, 2), ref) <= (2e-3 if _fp16_ops(ops, g, mode) else 1e-5)
    assert torch.equal(g.dgrad(dyd, wd, H, W), dx)  # deterministic
    sp = wd._dcs_sp
    del wd._dcs_sp
    try:
        dx0 = g.dgrad(dyd, wd, H, W)
    finally:
        wd._dcs_sp = sp
    assert _relmax(dx0.permute(0, 3, 1, 2), ref) <= (1e-5 if mode == "f16x3" else 2e-3)  # rows pass


@pytest.mark.parametrize("mode", ["f16x3", "f16"])
@pytest.mark.parametrize("cin,cout,N,H,W", [(256, 128, 2, 8, 64), (128, 64, 1, 17, 128), (128, 64, 1, 2, 256)])
def test_subpix_wgrad_vs_fp64(ops, mode, cin, cout, N, H, W):
    """dL/dW of the up-conv (the phase weight gradients folded onto the 3x3 taps) against float64
    autograd; strips of 64 source columns (the window kernel), row chunks not dividing H included."""
    ops.set_mma(mode)
    g = _geom(ops, cin, cout)
    x = rnd((N, cin, H, W), 87, "x").double()
    w = torch.from_numpy(prng.normal(88, "w", (cout, cin, 3, 3), 0, 0.05)).float().double().requires_grad_(True)
    dy = rnd((N, cout, 2 * H, 2 * W), 89, "dy").double()
    y = F.conv2d(F.interpolate(x, scale_factor=2, mode="nearest"), w, padding=1)
    (ref,) = torch.autograd.grad(y, w, dy)
    xd = x.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    dyd = dy.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    dw = g.wgrad(dyd, ops.Src.nhwc(xd))
    assert _relmax(dw, ref) <= (1e-5 if mode == "f16x3" else 2e-3)  # weight gradients in the step's mode


def _s2(ops, cin, cout):
    from modules.hip.lib import DCS_PAD_ZERO
    return ops.ConvGeom(cin, cout, 3, 2, (1, 1, 1, 1), DCS_PAD_ZERO)


@pytest.mark.parametrize("mode", ["f16x3", "f16"])
@pytest.mark.parametrize("cin,cout,N,H,W", [(64, 128, 2, 32, 32), (128, 256, 1, 64, 64), (64, 128, 1, 16, 256)])
def test_stride2_forward_stats_and_dgrad_vs_fp64(ops, mode, cin, cout, N, H, W):
    """The down-convs (stride-2 3x3 zero-pad-1) on the window phase kernels: forward + IN statistics
    over the source's parity classes, data gradient over dx's, against float64; the rows pass over the
    same packs (phase planes removed) to its own bound."""
    ops.set_mma(mode)
    g = _s2(ops, cin, cout)
    assert g.s2win
    x = rnd((N, cin, H, W), 91, "x").double().requires_grad_(True)
    w = torch.from_numpy(prng.normal(92, "w", (cout, cin, 3, 3), 0, 0.05)).float().double()
    ref = F.conv2d(x, w, stride=2, padding=1)
    dy = rnd(tuple(ref.shape), 93, "dy").double()
    (dref,) = torch.autograd.grad(ref, x, dy)
    ref = ref.detach()
    mean, var = ref.mean(dim=(2, 3)), ref.var(dim=(2, 3), unbiased=False)
    xd = x.detach().float().to(DEV).permute(0, 2, 3, 1).contiguous()
    wp, wd = g.pack_fwd(w.float().to(DEV)), g.pack_dgrad(w.float().to(DEV))
    assert getattr(wp, "_dcs_sp", None) is not None and getattr(wd, "_dcs_sp", None) is not None
    tol = 1e-5 if mode == "f16x3" else 2e-3  # the down-convs run in the step's operand mode
    y, st = g.forward_in_stats(ops.Src.nhwc(xd), wp, want_max=True)
    assert _relmax(y.permute(0, 3, 1, 2), ref) <= tol
    rstd = 1.0 / torch.sqrt(var + 1e-5)
    assert _relmax(st.scale, rstd) <= tol
    assert float((st.shift.double().cpu() + mean * rstd).abs().max()) <= tol * float((mean * rstd).abs().max() + 1)
    assert _relmax(st.xmax, ref.flatten(2).max(dim=2).values) <= tol
    assert torch.equal(g.forward(ops.Src.nhwc(xd), wp), y)
    dyd = dy.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    dx = g.dgrad(dyd, wd, H, W)
    assert _relmax(dx.permute(0, 3, 1, 2), dref) <= tol
    assert torch.equal(g.dgrad(dyd, wd, H, W), dx)  # deterministic
    rows_tol = 1e-5 if mode == "f16x3" else 2e-3
    for pk in (wp, wd):
        del pk._dcs_sp
    assert _relmax(g.forward(ops.Src.nhwc(xd), wp).permute(0, 3, 1, 2), ref) <= rows_tol
    assert _relmax(g.dgrad(dyd, wd, H, W).permute(0, 3, 1, 2), dref) <= rows_tol


@pytest.mark.parametrize("mode", ["f16x3", "f16"])
@pytest.mark.parametrize("cin,cout,N,H,W", [(64, 128, 2, 64, 64), (256, 512, 1, 64, 64), (128, 256, 1, 32, 256)])
def test_patchgan_layer_vs_fp64(ops, mode, cin, cout, N, H, W):
    """A PatchGAN layer (4x4 stride-2 zero-pad-1, modules/model.py:118-131) on the window phase kernels:
    forward with the previous layer's InstanceNorm + LeakyReLU as the staged prologue and the IN
    statistics of its output, and the data gradient, against float64."""
    from modules.hip.lib import ACT_LRELU, DCS_PAD_ZERO
    ops.set_mma(mode)
    g = ops.ConvGeom(cin, cout, 4, 2, (1, 1, 1, 1), DCS_PAD_ZERO)
    assert g.s2win
    y = rnd((N, cin, H, W), 94, "y").double()
    sc = (torch.from_numpy(prng.uniform(95, "sc", (N, cin), 0.5, 2.0))).double()
    sh = (torch.from_numpy(prng.uniform(95, "sh", (N, cin), -0.5, 0.5))).double()
    a = F.leaky_relu(y * sc[:, :, None, None] + sh[:, :, None, None], 0.2).requires_grad_(True)
    w = torch.from_numpy(prng.normal(96, "w", (cout, cin, 4, 4), 0, 0.05)).float().double()
    ref = F.conv2d(a, w, stride=2, padding=1)
    dy = rnd(tuple(ref.shape), 97, "dy").double()
    (dref,) = torch.autograd.grad(ref, a, dy)
    ref = ref.detach()
    mean, var = ref.mean(dim=(2, 3)), ref.var(dim=(2, 3), unbiased=False)
    yd = y.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    pro = (sc.float().to(DEV).contiguous(), sh.float().to(DEV).contiguous(), ACT_LRELU)
    wp, wd = g.pack_fwd(w.float().to(DEV)), g.pack_dgrad(w.float().to(DEV))
    assert getattr(wp, "_dcs_sp", None) is not None and getattr(wd, "_dcs_sp", None) is not None
    f16 = _fp16_ops(ops, g, mode)
    tol = 2e-3 if f16 else 1e-5
    out, st = g.forward_in_stats(ops.Src.nhwc(yd), wp, pro=pro)
    assert _relmax(out.permute(0, 3, 1, 2), ref) <= tol
    if f16:  # the prologue's activation rounded to fp16 (fp32 vs float64 activation: an ulp apart at most)
        ref16 = F.conv2d(_h(a.float()), _h(w), stride=2, padding=1)
        assert _relmax(out.permute(0, 3, 1, 2), ref16) <= 1e-4
        (dref16,) = torch.autograd.grad(F.conv2d(a, _h(w), stride=2, padding=1), a, _h(dy))
    rstd = 1.0 / torch.sqrt(var + 1e-5)
    assert _relmax(st.scale, rstd) <= tol
    assert float((st.shift.double().cpu() + mean * rstd).abs().max()) <= tol * float((mean * rstd).abs().max() + 1)
    assert torch.equal(g.forward(ops.Src.nhwc(yd), wp, pro=pro), out)
    dyd = dy.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    dx = g.dgrad(dyd, wd, H, W)
    assert _relmax(dx.permute(0, 3, 1, 2), dref) <= tol
    if f16:
        assert _relmax(dx.permute(0, 3, 1, 2), dref16) <= 2e-5
    rows_tol = 1e-5 if mode == "f16x3" else 2e-3
    for pk in (wp, wd):
        del pk._dcs_sp
    assert _relmax(g.forward(ops.Src.nhwc(yd), wp, pro=pro).permute(0, 3, 1, 2), ref) <= rows_tol
    assert _relmax(g.dgrad(dyd, wd, H, W).permute(0, 3, 1, 2), dref) <= rows_tol


@pytest.mark.parametrize("mode", ["f16x3", "f16"])
@pytest.mark.parametrize("k,cin,cout,N,H,W,pro", [(3, 64, 128, 1, 128, 128, False), (3, 128, 256, 2, 34, 128, False),
                                                  (4, 64, 128, 1, 64, 128, True), (4, 256, 512, 1, 32, 128, True)])
def test_stride2_wgrad_vs_fp64(ops, mode, k, cin, cout, N, H, W, pro):
    """dL/dW of a down-conv (3x3, the rolling class-window kernel) or a PatchGAN layer (4x4, with the
    IN + LeakyReLU prologue of its source; the x6 kernel) against float64 autograd; row chunks that do
    not divide the output rows included (Ho = 17)."""
    from modules.hip.lib import ACT_LRELU, DCS_PAD_ZERO
    ops.set_mma(mode)
    g = ops.ConvGeom(cin, cout, k, 2, (1, 1, 1, 1), DCS_PAD_ZERO)
    assert g.s2win
    y = rnd((N, cin, H, W), 98, "y").double()
    if pro:
        sc = torch.from_numpy(prng.uniform(99, "sc", (N, cin), 0.5, 2.0)).double()
        sh = torch.from_numpy(prng.uniform(99, "sh", (N, cin), -0.5, 0.5)).double()
        a = F.leaky_relu(y * sc[:, :, None, None] + sh[:, :, None, None], 0.2)
        prod = (sc.float().to(DEV).contiguous(), sh.float().to(DEV).contiguous(), ACT_LRELU)
    else:
        a, prod = y, None
    w = torch.from_numpy(prng.normal(100, "w", (cout, cin, k, k), 0, 0.05)).float().double().requires_grad_(True)
    out = F.conv2d(a, w, stride=2, padding=1)
    dy = rnd(tuple(out.shape), 101, "dy").double()
    (ref,) = torch.autograd.grad(out, w, dy)
    yd = y.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    dyd = dy.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    dw = g.wgrad(dyd, ops.Src.nhwc(yd), pro=prod)
    assert _relmax(dw, ref) <= (1e-5 if mode == "f16x3" else 2e-3)  # weight gradients in the step's mode


@pytest.mark.parametrize("layer", ["up2", "up1", "down1", "down2"])
def test_phase_dgrad_fused_in_backward(ops, layer):
    """The phase kernels' data gradient with the IN + ReLU backward's partial sums fused
    (dcs_phase_win_dgrad_inbwd -> in_act_backward_parts) equals the data gradient followed by the
    separate IN backward (in_act_backward), and the data gradient itself is bit-identical."""
    from modules.hip.lib import ACT_RELU, DCS_PAD_ZERO
    ops.set_mma("f16x3")
    cin, cout, H, W, g = {"up2": (128, 64, 32, 32, None), "up1": (256, 128, 16, 16, None),
                          "down1": (64, 128, 64, 64, 1), "down2": (128, 256, 32, 32, 1)}[layer]
    geo = _geom(ops, cin, cout) if g is None else _s2(ops, cin, cout)
    N = 2
    w = (rnd((cout, cin, 3, 3), 102, "w") * 0.05).float().to(DEV)
    wd = geo.pack_dgrad(w)
    assert getattr(wd, "_dcs_sp", None) is not None
    Ho, Wo = (2 * H, 2 * W) if g is None else (H // 2, W // 2)
    dy = rnd((N, Ho, Wo, cout), 103, "dy").float().to(DEV)
    y = rnd((N, H, W, cin), 104, "y").float().to(DEV)
    st = ops.in_stats(y)
    dx, parts, nch = geo.dgrad(dy, wd, H, W, inbwd=(y, st, ACT_RELU))
    assert parts is not None and nch > 0
    fused = ops.in_act_backward_parts(dx, y, st, ACT_RELU, parts, nch)
    dx0 = geo.dgrad(dy, wd, H, W)
    assert torch.equal(dx, dx0)
    sep = ops.in_act_backward(dx0, y, st, ACT_RELU)
    torch.testing.assert_close(fused, sep, rtol=1e-4, atol=1e-5 * float(sep.abs().max()))


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4, 5])
def test_subpix_pack_batched_bit_identical(ops, kind):
    ops.set_mma("f16x3")
    dgrad = kind in (1, 2, 5)
    if kind < 2:
        g = _geom(ops, 256, 128)
        w = (rnd((128, 256, 3, 3), 83, "w") * 0.05).float().to(DEV)
    elif kind < 4:
        g = _s2(ops, 128, 256)
        w = (rnd((256, 128, 3, 3), 83, "w") * 0.05).float().to(DEV)
    else:
        from modules.hip.lib import DCS_PAD_ZERO
        g = ops.ConvGeom(128, 256, 4, 2, (1, 1, 1, 1), DCS_PAD_ZERO)
        w = (rnd((256, 128, 4, 4), 83, "w") * 0.05).float().to(DEV)
    pack = g.pack_dgrad if dgrad else g.pack_fwd
    sp = [a.clone() for a in pack(w)._dcs_sp]
    w.mul_(1.0)
    ops.prepack([w])
    got = pack(w)._dcs_sp
    for a, b in zip(got, sp):
        assert torch.equal(a, b)
