"""MFMA operand modes of the convolution passes (rows: forward / data gradient; weight gradient) (include/ducosy_hip.h DCS_MMA_*) against a
float64 CPU reference of the same convolution, forward and data gradient, on every layer
geometry with a vectorised gather.  Tolerances (max |err| / max |ref|), written per mode:
  f32    exact fp32 MFMA                                  <= 1e-5
  bf16x3 hi/lo bf16 split, three products                 <= 5e-5   (~2^-16 per product)
  bf16   bf16 operands, f32 accumulation (config 5)       <= 2e-2   (~2^-9 per operand)
"""
import pytest
import torch

from oracle import prng
from test_gpu_ops import CONV_CASES, _geom, rnd, torch_conv

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = {"f32": 1e-5, "bf16x3": 5e-5, "bf16": 2e-2}
CASES = [c for c in CONV_CASES if c[0] % 16 == 0 and c[1] % 16 == 0]


def _relmax(a, b):
    return float((a.double().cpu() - b).abs().max() / b.abs().max())


@pytest.fixture
def ops():
    from modules.hip import ops as o
    yield o
    o.set_mma("f32")


@pytest.mark.parametrize("mode", ["bf16", "bf16x3", "f32"])
@pytest.mark.parametrize("case", CASES, ids=[f"c{c[0]}-{c[1]}k{c[2]}s{c[3]}u{c[6]}H{c[7]}" for c in CASES])
def test_conv_modes_vs_fp64(ops, mode, case):
    g, H = _geom(case)
    N = 2
    x = rnd((N, g.cin, H, H + 1), 11, "x").double()
    w = torch.from_numpy(prng.normal(12, "w", (g.cout, g.cin, g.k, g.k), 0, 0.05)).double()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = torch_conv(xr, wr, g)
    R = torch.from_numpy(prng.normal(13, "R", tuple(yr.shape))).double()
    (yr * R).sum().backward()

    ops.set_mma(mode)
    xd = x.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    wd = w.float().to(DEV)
    y = g.forward(ops.Src.nhwc(xd), g.pack_fwd(wd))
    assert _relmax(y.permute(0, 3, 1, 2), yr.detach()) <= TOL[mode]
    Rd = R.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    dx = g.dgrad(Rd, g.pack_dgrad(wd), H, H + 1)
    assert _relmax(dx.permute(0, 3, 1, 2), xr.grad) <= TOL[mode]
    dw = g.wgrad(Rd, ops.Src.nhwc(xd))
    assert _relmax(dw, wr.grad) <= TOL[mode]


def test_mode_switch_rejects_unknown(ops):
    with pytest.raises(ValueError):
        ops.set_mma("fp8")
