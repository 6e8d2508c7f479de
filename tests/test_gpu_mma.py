"""MFMA operand modes of the convolution passes (rows: forward / data gradient; weight gradient) (include/ducosy_hip.h DCS_MMA_*) against a
float64 CPU reference of the same convolution, forward and data gradient, on every layer
geometry with a vectorised gather.  Tolerances (max |err| / max |ref|), written per mode:
  f32    exact fp32 MFMA                                  <= 1e-5
  bf16x6 hi/mid/lo bf16 split, six products               <= 1e-5   (~2^-24 per product)
  f16x3  power-of-two scaled hi/lo fp16 split, 3 products <= 1e-5   (~2^-22 per operand)
  bf16x3 hi/lo bf16 split, three products                 <= 5e-5   (~2^-16 per product)
  f16    power-of-two scaled fp16 operands, one product   <= 3e-3   (~2^-11 per operand)
  bf16   bf16 operands, f32 accumulation (config 5)       <= 2e-2   (~2^-9 per operand)
"""
import pytest
import torch

from oracle import prng
from test_gpu_ops import CONV_CASES, _geom, rnd, torch_conv

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = {"f32": 1e-5, "bf16x6": 1e-5, "f16x3": 1e-5, "bf16x3": 5e-5, "f16": 3e-3, "bf16": 2e-2}
CASES = [c for c in CONV_CASES if c[0] % 16 == 0 and c[1] % 16 == 0]


def _relmax(a, b):
    return float((a.double().cpu() - b).abs().max() / b.abs().max())


@pytest.fixture
def ops():
    from modules.hip import ops as o
    prev = o.get_mma()
    yield o
    o.set_mma(prev)


@pytest.mark.parametrize("mode", ["bf16", "bf16x3", "bf16x6", "f16x3", "f16", "f32"])
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


def _errs(ops, mode, g, H, x, w, R):
    ops.set_mma(mode)
    xd = x.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    wd = w.float().to(DEV)
    y = g.forward(ops.Src.nhwc(xd), g.pack_fwd(wd)).permute(0, 3, 1, 2)
    Rd = R.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    dx = g.dgrad(Rd, g.pack_dgrad(wd), H, H + 1).permute(0, 3, 1, 2)
    dw = g.wgrad(Rd, ops.Src.nhwc(xd))
    return y, dx, dw


@pytest.mark.parametrize("case", CASES, ids=[f"c{c[0]}-{c[1]}k{c[2]}s{c[3]}u{c[6]}H{c[7]}" for c in CASES])
def test_bf16x6_error_matches_exact_f32(ops, case):
    """bf16x6 and f16x3 are fp32-class modes: against a float64 convolution of the SAME fp32
    operands, their max error (forward, data and weight gradient) is within 1.5x of the exact-fp32
    MFMA path's (all are dominated by the fp32 accumulation, not the operand split).  Errors are
    recorded in gpurun_out/x6_err.jsonl."""
    import json
    import os
    g, H = _geom(case)
    N = 2
    x = rnd((N, g.cin, H, H + 1), 21, "x").double()
    w = torch.from_numpy(prng.normal(22, "w", (g.cout, g.cin, g.k, g.k), 0, 0.05)).float().double()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = torch_conv(xr, wr, g)
    R = torch.from_numpy(prng.normal(23, "R", tuple(yr.shape))).float().double()
    (yr * R).sum().backward()
    e = {}
    for mode in ("f32", "bf16x6", "f16x3"):
        y, dx, dw = _errs(ops, mode, g, H, x, w, R)
        e[mode] = (_relmax(y, yr.detach()), _relmax(dx, xr.grad), _relmax(dw, wr.grad))
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/x6_err.jsonl", "a") as f:
        f.write(json.dumps({"case": list(case), **e}) + "\n")
    for k in range(3):  # forward, data gradient, weight gradient
        assert e["bf16x6"][k] <= 1.5 * e["f32"][k] + 1e-7, e
        assert e["f16x3"][k] <= 1.5 * e["f32"][k] + 1e-7, e


@pytest.mark.parametrize("scale", [1e-9, 1e-3, 1e4])
@pytest.mark.parametrize("case", CASES[:3], ids=[f"c{c[0]}-{c[1]}k{c[2]}s{c[3]}u{c[6]}H{c[7]}" for c in CASES[:3]])
def test_f16x3_scale_invariant(ops, case, scale):
    """f16x3 scales each operand by a power of two from its range record, so the relative error
    does not depend on the operands' magnitude (gradients of 1e-9, activations of 1e4; fp16 alone
    covers 6e-8 .. 65504).  Heavy-tailed data (one in 10^4 values x100) keeps the bar."""
    g, H = _geom(case)
    N = 2
    x = rnd((N, g.cin, H, H + 1), 41, "x").double() * scale
    x.view(-1)[::9973] *= 100.0
    w = torch.from_numpy(prng.normal(42, "w", (g.cout, g.cin, g.k, g.k), 0, 0.05)).float().double()
    xr = x.float().double().clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = torch_conv(xr, wr, g)
    R = (torch.from_numpy(prng.normal(43, "R", tuple(yr.shape))).double() * scale).float().double()
    (yr * R).sum().backward()
    y, dx, dw = _errs(ops, "f16x3", g, H, xr.detach(), w, R)
    assert _relmax(y, yr.detach()) <= TOL["f16x3"]
    assert _relmax(dx, xr.grad) <= TOL["f16x3"]
    assert _relmax(dw, wr.grad) <= TOL["f16x3"]


@pytest.mark.parametrize("mode", ["f32", "bf16x6", "bf16x3", "f16x3"])
def test_modes_deterministic(ops, mode):
    """Every MFMA mode is run-to-run deterministic (bit-identical forward and data gradient),
    also with other work in flight on a second stream."""
    ops.set_mma(mode)
    side = torch.cuda.Stream()
    for case in CASES:
        g, H = _geom(case)
        x = rnd((2, g.cin, H, H + 1), 31, "x").float().to(DEV).permute(0, 2, 3, 1).contiguous()
        w = torch.from_numpy(prng.normal(32, "w", (g.cout, g.cin, g.k, g.k), 0, 0.05)).float().to(DEV)
        pf, pd = g.pack_fwd(w), g.pack_dgrad(w)
        outs = []
        for rep in range(4):
            if rep % 2:
                with torch.cuda.stream(side):
                    g.forward(ops.Src.nhwc(x), pf)
            y = g.forward(ops.Src.nhwc(x), pf)
            dx = g.dgrad(y.contiguous(), pd, H, H + 1)
            outs.append((y.clone(), dx.clone()))
        torch.cuda.synchronize()
        for y, dx in outs[1:]:
            assert torch.equal(y, outs[0][0]), (mode, case)
            assert torch.equal(dx, outs[0][1]), (mode, case)


@pytest.mark.parametrize("mode", ["f16x3", "f16"])
@pytest.mark.parametrize("case", [(3, 64, 7, 1, (3, 3, 3, 3), "reflect", 1, 40), (1, 64, 4, 2, (1, 1, 1, 1), "zero", 1, 48)],
                         ids=["stem", "d0"])
def test_wgrad_4ch_source_vs_fp64(ops, mode, case):
    """Weight gradients over the packed 4-channel NHWC source (the stem's image + masks, PatchGAN
    layer 0) on the fp16 x6 kernel (conv_wgrad_x6_kernel<., ., V4>) against float64."""
    g, H = _geom(case)
    N = 2
    x = rnd((N, g.cin, H, H + 1), 51, "x").double()
    w = torch.from_numpy(prng.normal(52, "w", (g.cout, g.cin, g.k, g.k), 0, 0.05)).double()
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    yr = torch_conv(xr, wr, g)
    R = torch.from_numpy(prng.normal(53, "R", tuple(yr.shape))).float().double()
    (yr * R).sum().backward()
    ops.set_mma(mode)
    x4 = ops.pack_nhwc4(x.float().to(DEV)[:, :1].contiguous(), x.float().to(DEV)[:, 1:].contiguous()
                        if g.cin > 1 else None)
    Rd = R.float().to(DEV).permute(0, 2, 3, 1).contiguous()
    dw = g.wgrad(Rd, ops.Src.nhwc(x4))
    assert _relmax(dw, wr.grad) <= TOL[mode]
