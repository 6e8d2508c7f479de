"""The f16x3 window kernel of the residual-block convolutions (csrc/conv_win.hip;
modules/model.py:72-80) against float64 references of the same fp32 operands:
  * forward (reflection pad 1) + the InstanceNorm statistics of its output (scale / shift / max /
    argmax from the epilogue partials) at W = 16, 32, 64, 128;
  * the data gradient onto the reflection-padded input (interior by the window pass, the padded
    grid's ring by the rows pass, folded onto the border), with and without the residual addend;
  * equality of bar with the rows pass it replaces: the same fp32-class bound (max error / max |ref|
    <= 1e-5) and within 1.5x of the exact-f32 MFMA path's error.
Tolerances written per check below."""
import ctypes

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
    prev, prev_win = o.get_mma(), o._WIN
    yield o
    o.set_mma(prev)
    o._WIN = prev_win


def _geom(ops, cin=256, cout=256):
    from modules.hip.lib import DCS_PAD_REFLECT
    return ops.ConvGeom(cin, cout, 3, 1, (1, 1, 1, 1), DCS_PAD_REFLECT)


@pytest.mark.parametrize("N,H,W", [(2, 16, 16), (1, 32, 32), (2, 16, 64), (1, 8, 128)])
def test_win_forward_and_stats_vs_fp64(ops, N, H, W):
    ops.set_mma("f16x3")
    g = _geom(ops)
    assert g.win
    x = rnd((N, 256, H, W), 51, "x").double()
    w = torch.from_numpy(prng.normal(52, "w", (256, 256, 3, 3), 0, 0.05)).float().double()
    ref = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), w)
    mean = ref.mean(dim=(2, 3))
    var = ref.var(dim=(2, 3), unbiased=False)
    xd = x.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    wp = g.pack_fwd(w.float().to(DEV))
    assert getattr(wp, "_dcs_h3", None) is not None
    ops.PROBE.reset()
    y, st = g.forward_in_stats(ops.Src.nhwc(xd), wp, want_max=True)
    assert _relmax(y.permute(0, 3, 1, 2), ref) <= 1e-5
    rstd = 1.0 / torch.sqrt(var + 1e-5)
    assert _relmax(st.scale, rstd) <= 1e-5
    assert float((st.shift.double().cpu() + mean * rstd).abs().max()) <= 1e-5 * float((mean * rstd).abs().max() + 1)
    mx = ref.flatten(2).max(dim=2)
    assert _relmax(st.xmax, mx.values) <= 1e-5
    # argmax: the first maximum; where two values tie to within rounding either index is right
    am = st.xargmax.cpu().long()
    got_at = ref.flatten(2).gather(2, am[..., None])[..., 0]
    assert float((got_at - mx.values).abs().max()) <= 1e-5 * float(mx.values.abs().max())


@pytest.mark.parametrize("addend", [False, True])
@pytest.mark.parametrize("N,H,W", [(2, 16, 16), (1, 16, 128), (5, 32, 32), (3, 16, 64), (2, 8, 128)])
def test_win_dgrad_reflect_vs_fp64(ops, N, H, W, addend):
    """The reflect-pad data gradient: interior by the window kernel, the padded grid's ring by
    ring16_kernel (ring segments over the batch in 64-position tiles: the sizes here leave partial
    tiles and tiles that straddle images), folded onto the border; against float64 at 1e-5."""
    ops.set_mma("f16x3")
    g = _geom(ops)
    x = rnd((N, 256, H, W), 61, "x").double().requires_grad_(True)
    w = torch.from_numpy(prng.normal(62, "w", (256, 256, 3, 3), 0, 0.05)).float().double()
    y = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), w)
    R = torch.from_numpy(prng.normal(63, "R", tuple(y.shape))).float().double()
    A = rnd((N, 256, H, W), 64, "A").double() if addend else None
    (y * R).sum().backward()
    ref = x.grad + (A if addend else 0)
    Rd = R.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    Ad = A.float().to(DEV).permute(0, 2, 3, 1).contiguous() if addend else None
    wd = g.pack_dgrad(w.float().to(DEV))
    assert getattr(wd, "_dcs_h3", None) is not None
    dx = g.dgrad(Rd, wd, H, W, addend=Ad)
    assert _relmax(dx.permute(0, 3, 1, 2), ref) <= 1e-5


def test_win_matches_rows_pass_error(ops):
    """The window pass and the rows pass it replaces (both f16x3) against the exact-f32 path's error
    vs float64: within 1.5x (fp32-class), forward and data gradient."""
    N, H, W = 2, 32, 32
    g = _geom(ops)
    x = rnd((N, 256, H, W), 71, "x").double().requires_grad_(True)
    w = torch.from_numpy(prng.normal(72, "w", (256, 256, 3, 3), 0, 0.05)).float().double()
    y = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), w)
    R = torch.from_numpy(prng.normal(73, "R", tuple(y.shape))).float().double()
    (y * R).sum().backward()
    xd = x.detach().float().to(DEV).permute(0, 2, 3, 1).contiguous()
    Rd = R.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    err = {}
    for tag, mode, win in (("f32", "f32", False), ("rows", "f16x3", False), ("win", "f16x3", True)):
        ops.set_mma(mode)
        ops._WIN = win
        wd = w.float().to(DEV)
        yy, _ = g.forward_in_stats(ops.Src.nhwc(xd), g.pack_fwd(wd))
        dx = g.dgrad(Rd, g.pack_dgrad(wd), H, W)
        err[tag] = (_relmax(yy.permute(0, 3, 1, 2), y.detach()), _relmax(dx.permute(0, 3, 1, 2), x.grad))
    for k in range(2):
        assert err["win"][k] <= 1.5 * err["f32"][k] + 1e-7, err
        assert err["rows"][k] <= 1.5 * err["f32"][k] + 1e-7, err


def test_win_ok_rejects_other_geometries(ops):
    from modules.hip import lib
    ops.set_mma("f16x3")
    g = _geom(ops)
    x = torch.zeros(1, 9, 9, 256, device=DEV)  # 256 % 9 != 0: the rows pass keeps these
    d = g._desc_fwd(ops.Src.nhwc(x), 2304, 0, 0)
    ops._set_mma(d, x, None, torch.zeros(512, device=DEV))
    assert lib.query("dcs_conv3_win_ok", ctypes.byref(d), 0) == 0


@pytest.mark.parametrize("N,H,W", [(2, 16, 64), (1, 20, 64), (1, 8, 128), (1, 32, 128)])
def test_win_wgrad_vs_fp64(ops, N, H, W):
    """The rolling-window weight gradient (csrc/conv_win.hip wgrad3_win_h3_kernel: 64-pixel strips,
    row chunks of 8..H rows, reflection halo) against float64: max error / max |ref| <= 1e-5, and
    within 1.5x of the exact-f32 MFMA path's error (fp32-class), bit-identical on a second run."""
    from modules.hip import lib
    g = _geom(ops)
    x = rnd((N, 256, H, W), 81, "x").double()
    w = torch.from_numpy(prng.normal(82, "w", (256, 256, 3, 3), 0, 0.05)).float().double().requires_grad_(True)
    y = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), w)
    R = torch.from_numpy(prng.normal(83, "R", tuple(y.shape))).float().double()
    (y * R).sum().backward()
    xd = x.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    Rd = R.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    ops.set_mma("f16x3")
    d = g._desc_fwd(ops.Src.nhwc(xd), 0, 0, 0)
    ops._set_mma(d, Rd, None, ops.range_rec(xd))
    assert lib.query("dcs_conv_wgrad_workspace_size", ctypes.byref(d)) >= N * (W // 64) * 256 * 2304 * 4
    dw = g.wgrad(Rd, ops.Src.nhwc(xd))
    e_win = _relmax(dw, w.grad)
    assert e_win <= 1e-5, e_win
    assert torch.equal(dw, g.wgrad(Rd, ops.Src.nhwc(xd)))
    ops.set_mma("f32")
    e_f32 = _relmax(g.wgrad(Rd, ops.Src.nhwc(xd)), w.grad)
    assert e_win <= 1.5 * e_f32 + 1e-7, (e_win, e_f32)


@pytest.mark.parametrize("N,H,W", [(2, 16, 64), (1, 16, 128)])
def test_win_f16_mode_vs_fp64(ops, N, H, W):
    """BASELINE config 5's fp16 MFMA path (DCS_MMA_F16: the window kernels with the hi planes only,
    one product): forward, data gradient and weight gradient within 3e-3 of float64 (fp16 operands:
    2^-11 per operand), and the f16x3 result within 1e-5 on the same operands."""
    g = _geom(ops)
    x = rnd((N, 256, H, W), 91, "x").double().requires_grad_(True)
    w = torch.from_numpy(prng.normal(92, "w", (256, 256, 3, 3), 0, 0.05)).float().double().requires_grad_(True)
    y = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), w)
    R = torch.from_numpy(prng.normal(93, "R", tuple(y.shape))).float().double()
    (y * R).sum().backward()
    xd = x.detach().float().to(DEV).permute(0, 2, 3, 1).contiguous()
    Rd = R.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    for mode, tol in (("f16", 3e-3), ("f16x3", 1e-5)):
        ops.set_mma(mode)
        wd = w.detach().float().to(DEV)
        yy, _ = g.forward_in_stats(ops.Src.nhwc(xd), g.pack_fwd(wd))
        dx = g.dgrad(Rd, g.pack_dgrad(wd), H, W)
        dw = g.wgrad(Rd, ops.Src.nhwc(xd))
        errs = (_relmax(yy.permute(0, 3, 1, 2), y.detach()), _relmax(dx.permute(0, 3, 1, 2), x.grad),
                _relmax(dw, w.grad))
        assert max(errs) <= tol, (mode, errs)


@pytest.mark.parametrize("N,H,W", [(1, 18, 64), (2, 16, 64), (1, 20, 128), (1, 9, 64)])
def test_win_wgrad_f16_vs_fp64(ops, N, H, W):
    """The f16 mode's weight gradient (wgrad3_win16_kernel<1>: two image rows per barrier, the next
    two staged through the second) over row chunks with an odd row count (H 18: two chunks of 9, H 9:
    one) and several strips: within 3e-3 of float64 and bit-identical on a second run."""
    g = _geom(ops)
    x = rnd((N, 256, H, W), 121, "x").double()
    w = torch.from_numpy(prng.normal(122, "w", (256, 256, 3, 3), 0, 0.05)).float().double().requires_grad_(True)
    y = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), w)
    R = torch.from_numpy(prng.normal(123, "R", tuple(y.shape))).float().double()
    (y * R).sum().backward()
    xd = x.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    Rd = R.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    ops.set_mma("f16")
    dw = g.wgrad(Rd, ops.Src.nhwc(xd))
    e = _relmax(dw, w.grad)
    assert e <= 3e-3, e
    assert torch.equal(dw, g.wgrad(Rd, ops.Src.nhwc(xd)))


@pytest.mark.parametrize("N,H,W", [(2, 16, 16), (1, 16, 128)])
def test_win_dgrad_inbwd_matches_separate_pass(ops, N, H, W):
    """The InstanceNorm backward of a = relu(IN(y)) with its partial sums fused into the window data
    gradient that produces da (dcs_conv_dgrad_reflect_win_inbwd: tile epilogue + ring fold) against the
    separate partial-sum pass on the same da (dcs_in_act_backward): dx bit-identical (same kernels),
    dy within 1e-5 of max |dy| (the sums run in a different order), and against float64."""
    from modules.hip.lib import ACT_RELU
    ops.set_mma("f16x3")
    g = _geom(ops)
    y = rnd((N, 256, H, W), 111, "y").float().to(DEV).permute(0, 2, 3, 1).contiguous()
    st = ops.in_stats(y)
    w = torch.from_numpy(prng.normal(112, "w", (256, 256, 3, 3), 0, 0.05)).float().to(DEV)
    R = torch.from_numpy(prng.normal(113, "R", (N, 256, H, W))).float().to(DEV).permute(0, 2, 3, 1).contiguous()
    wd = g.pack_dgrad(w)
    da_f, parts, nch = g.dgrad(R, wd, H, W, inbwd=(y, st, ACT_RELU))
    assert parts is not None and nch == H * W // 256 + 64
    dy_f = ops.in_act_backward_parts(da_f, y, st, ACT_RELU, parts, nch)
    da_s = g.dgrad(R, wd, H, W)
    assert torch.equal(da_f, da_s)
    dy_s = ops.in_act_backward(da_s, y, st, ACT_RELU)
    assert _relmax(dy_f, dy_s.double().cpu()) <= 1e-5
    # float64 IN backward of the same da
    yd = y.double().cpu().requires_grad_(True)
    m = yd.mean(dim=(1, 2), keepdim=True)
    v = yd.var(dim=(1, 2), unbiased=False, keepdim=True)
    a = torch.relu((yd - m) / torch.sqrt(v + 1e-5))
    (a * da_s.double().cpu()).sum().backward()
    assert _relmax(dy_f, yd.grad) <= 1e-4


@pytest.mark.parametrize("mode", ["f16x3", "f16"])
def test_win_batch_vs_per_image_bit_identical(ops, mode):
    """A full-size batch (N = 3 at 128 x 128 x 256: 384 jobs, more than the GPU has CUs) against the same
    convs one image at a time: bit-identical outputs and IN statistics (forward), data gradients with
    the residual addend bit-identical, the reflection ring included (ring16_kernel sums each ring position
    in one fixed order whatever the batch; the rows pass it replaced split K by the batch size), and the
    data gradient with the InstanceNorm-backward partial sums in its epilogue (the training step's form)
    equal to the one without them."""
    ops.set_mma(mode)
    g = _geom(ops)
    N, H, W = 3, 128, 128
    xd = rnd((N, 256, H, W), 71, "x").float().to(DEV).permute(0, 2, 3, 1).contiguous()
    w = torch.from_numpy(prng.normal(72, "w", (256, 256, 3, 3), 0, 0.05)).float().to(DEV)
    wp = g.pack_fwd(w)
    y, st = g.forward_in_stats(ops.Src.nhwc(xd), wp, want_max=True)
    Rd = rnd((N, 256, H, W), 73, "R").float().to(DEV).permute(0, 2, 3, 1).contiguous()
    Ad = rnd((N, 256, H, W), 74, "A").float().to(DEV).permute(0, 2, 3, 1).contiguous()
    wd = g.pack_dgrad(w)
    dx = g.dgrad(Rd, wd, H, W, addend=Ad)
    for i in range(N):
        yi, sti = g.forward_in_stats(ops.Src.nhwc(xd[i:i + 1].contiguous()), wp, want_max=True)
        assert torch.equal(y[i:i + 1], yi), (mode, i)
        for a, b in ((st.scale, sti.scale), (st.shift, sti.shift), (st.xmax, sti.xmax), (st.xargmax, sti.xargmax)):
            assert torch.equal(a[i:i + 1], b), (mode, i)
        dxi = g.dgrad(Rd[i:i + 1].contiguous(), wd, H, W, addend=Ad[i:i + 1].contiguous())
        assert torch.equal(dx[i:i + 1], dxi), (mode, i)
    # the data gradient with the InstanceNorm-backward partial sums in its epilogue (the training step's
    # form; zero padding, whose window halo must survive the epilogue's LDS use): the same da as
    # without them, and the IN backward from the fused sums within 1e-5 of the separate pass
    from modules.hip.lib import ACT_RELU
    st_y = ops.in_stats(y)
    da_f, parts, nch = g.dgrad(Rd, wd, H, W, inbwd=(y, st_y, ACT_RELU))
    da_s = g.dgrad(Rd, wd, H, W)
    assert parts is not None and torch.equal(da_f, da_s), mode
    dy_f = ops.in_act_backward_parts(da_f, y, st_y, ACT_RELU, parts, nch)
    dy_s = ops.in_act_backward(da_s, y, st_y, ACT_RELU)
    assert _relmax(dy_f, dy_s.double().cpu()) <= 1e-5, mode
