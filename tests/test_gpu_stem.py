"""The Generator stem on its MFMA kernel (csrc/conv_stem.hip dcs_stem_fwd, the fp16 operand modes):
ReflectionPad2d(3) + Conv2d(cin, 64, 7) over the packed image and mask planes (modules/model.py:96-98)
and the InstanceNorm statistics of its output, against float64 on the same inputs, and against the
generic rows pass it replaces.  f16x3: output max |err| / max |ref| <= 2e-6, IN scale / shift within
1e-5; f16: 3e-3 / 3e-3 (the f16 mode runs the stem kernels on fp16 operands since round 6, ops._FIXED_F16X3)."""
import pytest
import torch
import torch.nn.functional as F

from oracle import prng
from test_gpu_ops import rnd

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _relmax(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max())


@pytest.mark.parametrize("N,H,W,cin", [(2, 64, 64, 3), (1, 40, 200, 2), (1, 512, 512, 3), (2, 7, 9, 3)])
@pytest.mark.parametrize("mode,tol", [("f16x3", 2e-6), ("f16", 3e-3)])
def test_stem_vs_fp64(N, H, W, cin, mode, tol):
    from modules.hip import ops
    from modules.hip.lib import DCS_PAD_REFLECT
    prev, prev_stem = ops.get_mma(), ops._STEM
    ops.set_mma(mode)
    try:
        g = ops.ConvGeom(cin, 64, 7, 1, (3, 3, 3, 3), DCS_PAD_REFLECT)
        img = rnd((N, 1, H, W), 71, "x").float().to(DEV)
        mk = (rnd((N, cin - 1, H, W), 72, "m", 0.0, 1.0) > 0.7).float().to(DEV)
        w = torch.from_numpy(prng.normal(73, "w", (64, cin, 7, 7), 0, 0.02)).float().to(DEV)
        x4 = ops.pack_nhwc4(img, mk)
        src = ops.Src.nhwc(x4)
        pk = g.pack_fwd(w, cin_pad=4)
        y, st = g.forward_in_stats(src, pk)
        x = torch.cat([img, mk], 1).double().cpu()
        ref = F.conv2d(F.pad(x, (3, 3, 3, 3), mode="reflect"), w.double().cpu()).permute(0, 2, 3, 1)
        e = _relmax(y.cpu(), ref)
        m = ref.mean((1, 2))
        rstd = 1.0 / torch.sqrt(ref.var((1, 2), unbiased=False) + 1e-5)
        e_sc = float(((st.scale.double().cpu() - rstd).abs() / rstd).max())
        e_sh = float((st.shift.double().cpu() + m * rstd).abs().max())
        ops._STEM = False
        y_rows, st_rows = g.forward_in_stats(src, pk)
        print(mode, (N, H, W, cin), "stem", e, "scale", e_sc, "shift", e_sh, "rows pass", _relmax(y_rows.cpu(), ref))
        assert e <= tol, e
        stol = 1e-5 if mode == "f16x3" else 3e-3
        assert e_sc <= stol and e_sh <= stol, (e_sc, e_sh)
        assert not torch.equal(y, y_rows)  # the stem kernel ran
        ops._STEM = True
        torch.testing.assert_close(g.forward_in_stats(src, pk)[0], y, rtol=0, atol=0)  # deterministic
        torch.testing.assert_close(g.forward(src, pk), y, rtol=0, atol=0)  # forward() takes the same kernel
    finally:
        ops.set_mma(prev)
        ops._STEM = prev_stem


@pytest.mark.parametrize("N,H,W,cin", [(2, 64, 64, 3), (1, 40, 200, 2), (1, 512, 512, 3), (2, 7, 9, 3)])
@pytest.mark.parametrize("mode,tol", [("f16x3", 5e-6), ("f16", 5e-3)])
def test_stem_wgrad_vs_fp64(N, H, W, cin, mode, tol):
    """dcs_stem_wgrad: dW of the stem against float64, and against the x6 weight-gradient kernel."""
    from modules.hip import ops
    from modules.hip.lib import DCS_PAD_REFLECT
    prev, prev_stem = ops.get_mma(), ops._STEM
    ops.set_mma(mode)
    try:
        g = ops.ConvGeom(cin, 64, 7, 1, (3, 3, 3, 3), DCS_PAD_REFLECT)
        img = rnd((N, 1, H, W), 81, "x").float().to(DEV)
        mk = (rnd((N, cin - 1, H, W), 82, "m", 0.0, 1.0) > 0.7).float().to(DEV)
        dy = (rnd((N, H, W, 64), 83, "dy") * 1e-2).float().to(DEV)
        src = ops.Src.nhwc(ops.pack_nhwc4(img, mk))
        x = torch.cat([img, mk], 1).double().cpu()
        ref = torch.nn.grad.conv2d_weight(F.pad(x, (3, 3, 3, 3), mode="reflect"), (64, cin, 7, 7),
                                          dy.double().cpu().permute(0, 3, 1, 2))
        dw = g.wgrad(dy, src)
        ops._STEM = False
        dw_x6 = g.wgrad(dy, src)
        e, e6 = _relmax(dw.cpu(), ref), _relmax(dw_x6.cpu(), ref)
        print(mode, (N, H, W, cin), "stem wgrad", e, "x6", e6)
        assert e <= tol, (e, e6)
        assert not torch.equal(dw, dw_x6)
        ops._STEM = True
        torch.testing.assert_close(g.wgrad(dy, src), dw, rtol=0, atol=0)
    finally:
        ops.set_mma(prev)
        ops._STEM = prev_stem
