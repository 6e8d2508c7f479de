"""Pre-split fp16 weight planes of the f16x3 / f16 rows pass (dcs_pack_split_h3, dcs_conv_desc.b_h3):
staging B from the planes gives bit-identical outputs to splitting the fp32 pack at staging (the
split is the same function of the same exponent), for the layer shapes that run the rows pass —
stride-2 forward (down1), sub-pixel up-convs (up1: 128-column tiles, up2: 64-column tiles), the
PatchGAN IN + LeakyReLU gather (d1) — and their data gradients (stride-2 parity classes, the
sub-pixel adjoint).  Zeroing the planes must change the output: the planes path ran.  (The up- and
down-convolutions run on the window phase kernels in production, csrc/conv_subpix.hip; their rows pass
stays the path for the shapes those do not tile.)"""
import pytest
import torch

from test_gpu_ops import rnd

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("mode", ["f16x3", "f16"])
@pytest.mark.parametrize("name", ["down1", "up1", "up2", "d1"])
def test_presplit_b_bit_identical(mode, name):
    from modules.hip import ops
    from modules.hip.lib import ACT_LRELU, DCS_PAD_ZERO
    from modules.hip.ops import ConvGeom, Src
    geoms = {
        "down1": (ConvGeom(64, 128, 3, 2, (1, 1, 1, 1)), 64, False),
        "up1": (ConvGeom(256, 128, 3, 1, (1, 1, 1, 1), DCS_PAD_ZERO, up=2), 32, False),
        "up2": (ConvGeom(128, 64, 3, 1, (1, 1, 1, 1), DCS_PAD_ZERO, up=2), 64, False),
        "d1": (ConvGeom(64, 128, 4, 2, (1, 1, 1, 1)), 64, True),
    }
    g, H, lrelu = geoms[name]
    prev = ops.get_mma()
    ops.set_mma(mode)
    try:
        N = 2
        x = rnd((N, H, H, g.cin), 61, name + "x").float().to(DEV)
        w = (rnd((g.cout, g.cin, g.k, g.k), 62, name + "w") * 0.05).float().to(DEV)
        pro = None
        if lrelu:
            st = ops.in_stats(x)
            pro = (st.scale, st.shift, ACT_LRELU)
        Ho, Wo = g.out_hw(H, H)
        dy = rnd((N, Ho, Wo, g.cout), 63, name + "dy").float().to(DEV)
        pk, pd = g.pack_fwd(w), g.pack_dgrad(w)
        assert hasattr(pk, "_dcs_bh3") and hasattr(pd, "_dcs_bh3")
        for p_ in (pk, pd):  # the rows pass (the window phase kernels take these layers in production)
            if hasattr(p_, "_dcs_sp"):
                del p_._dcs_sp
        y1 = g.forward(Src.nhwc(x), pk, pro=pro)
        d1 = g.dgrad(dy, pd, H, H)
        bh_f, bh_d = pk._dcs_bh3, pd._dcs_bh3
        del pk._dcs_bh3, pd._dcs_bh3
        y0 = g.forward(Src.nhwc(x), pk, pro=pro)
        d0 = g.dgrad(dy, pd, H, H)
        torch.testing.assert_close(y1, y0, rtol=0, atol=0)
        torch.testing.assert_close(d1, d0, rtol=0, atol=0)
        bh_f[1].zero_()
        pk._dcs_bh3 = bh_f
        assert not torch.equal(g.forward(Src.nhwc(x), pk, pro=pro), y0)
        bh_d[1].zero_()
        pd._dcs_bh3 = bh_d
        assert not torch.equal(g.dgrad(dy, pd, H, H), d0)
    finally:
        ops.set_mma(prev)
