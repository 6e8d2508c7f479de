"""The pre-split LDS-DMA bf16x6 residual conv (csrc/conv_x6p.hip) against the split-in-the-gather
bf16x6 rows kernel of conv.hip and against float64.

Both kernels issue the same six bf16 products per operand pair into two-level fp32 chains
(inner chains of 128 k) from the same hi/mid/lo split; the rows kernel walks K in 16-channel
slices, so the two are compared through their error against float64.  Cases: the forward (reflection padding 1) and the stride-1 data
gradient (zero padding 2 onto the padded grid), a pixel count that is not a multiple of the
128-row tile, and more than one image.
"""
import numpy as np
import pytest
import torch

from oracle import prng

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _res():
    from modules.hip.lib import DCS_PAD_REFLECT
    from modules.hip.ops import ConvGeom
    return ConvGeom(256, 256, 3, 1, (1, 1, 1, 1), DCS_PAD_REFLECT)


def _run(x6p, fn):
    """fn(packed forward weights, packed dgrad weights) with the x6p pass on, or with conv.hip's
    bf16x6 rows kernel in the same (tap-major) K order."""
    from modules.hip import ops
    prev_mode, prev, prev_ks = ops.get_mma(), ops._X6P, ops._KSLICE
    ops.set_mma("bf16x6")
    ops._X6P, ops._KSLICE = x6p, False
    try:
        out = fn()
        torch.cuda.synchronize()
        return out
    finally:
        ops._X6P, ops._KSLICE = prev, prev_ks
        ops.set_mma(prev_mode)


@pytest.mark.parametrize("n,h", [(2, 16), (3, 13), (1, 32)])
def test_x6p_forward_and_dgrad_vs_float64(n, h):
    """The x6p pass (tap-major K order) and conv.hip's bf16x6 rows kernel (which walks its K in
    16-channel slices, so its chains hold different terms) against a float64 forward and data
    gradient: the x6p error stays within 1.5x of the rows kernel's (the fp32-class bar of
    tests/test_gpu_mma.py)."""
    from modules.hip import ops
    g = _res()
    x = torch.from_numpy(prng.normal(61, f"x{n}{h}", (n, h, h, 256))).float().to(DEV)
    w = torch.from_numpy(prng.normal(62, "w", (256, 256, 3, 3), 0, 0.02)).float().to(DEV)
    dy = torch.from_numpy(prng.normal(63, f"dy{n}{h}", (n, h, h, 256))).float().to(DEV)
    d = g._desc_fwd(ops.Src.nhwc(x), 2304, 0, 0)
    d.mma, d.korder = 6, 0
    from modules.hip import lib
    import ctypes
    assert lib.query("dcs_conv_rows_x6p_ok", ctypes.byref(d)) == 1
    f_new = _run(True, lambda: g.forward(ops.Src.nhwc(x), g.pack_fwd(w)))
    f_old = _run(False, lambda: g.forward(ops.Src.nhwc(x), g.pack_fwd(w)))
    b_new = _run(True, lambda: g.dgrad(dy, g.pack_dgrad(w), h, h))
    b_old = _run(False, lambda: g.dgrad(dy, g.pack_dgrad(w), h, h))
    xd = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    ref = torch.nn.functional.conv2d(torch.nn.functional.pad(xd, (1, 1, 1, 1), mode="reflect"), w.double())
    ref.backward(dy.double().permute(0, 3, 1, 2))
    gref = xd.grad

    def err(a, r):
        return float((a.double().permute(0, 3, 1, 2) - r).abs().max() / r.abs().max())

    for new, old, r in ((f_new, f_old, ref.detach()), (b_new, b_old, gref)):
        e_new, e_old = err(new, r), err(old, r)
        assert e_new < 2e-6 and e_new <= 1.5 * e_old + 1e-7, (e_new, e_old)


def test_split_x6_planes():
    """dcs_split_x6: v = hi + mid + lo exactly representable pieces, interleaved per 8 elements."""
    from modules.hip import ops
    x = torch.from_numpy(prng.normal(64, "s", (4096,))).float().to(DEV) * 3.7
    sp = ops.split_x6(x).view(-1, 3, 8).view(torch.bfloat16).float()  # [groups][plane][8]
    rec = (sp[:, 0] + sp[:, 1] + sp[:, 2]).reshape(-1)
    err = (rec - x).abs() / x.abs().clamp_min(1e-30)
    assert float(err.max()) < 2 ** -22
    hi = x.view(-1, 8).to(torch.bfloat16).float()
    assert torch.equal(sp[:, 0], hi)
