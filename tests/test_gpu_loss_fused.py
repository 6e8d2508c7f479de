"""The fused G-step loss kernel (include/ducosy_hip.h dcs_gen_loss_fused; the north star's fused
cycle / identity / SSIM / gradient / contrast-loss kernel) against the per-term loss kernels,
which tests/test_gpu_ops.py and tests/test_gpu_fullsize.py pin to the oracle (the reference's
trainer.py:22-184, 347-351 and pytorch_msssim restated).  Values: relative 1e-5; gradient planes:
max |err| / max |ref| <= 1e-5 (the fused kernel sums the terms' d/dpred in one expression per
pixel, the per-term path in separate planes)."""
import pytest
import torch

from oracle import prng

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _u(seed, tag, shape, lo=-1.0, hi=1.0):
    return torch.from_numpy(prng.uniform(seed, tag, shape, lo, hi)).float().to(DEV)


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("shape", [(2, 80, 72), (3, 64, 64), (1, 45, 130)])
def test_fused_loss_matches_per_term_kernels(shape):
    from modules.hip import ops
    from modules.hip.lib import GL_CA, GL_GRAD, GL_L1, GL_MSEC, GL_SSIM
    N, H, W = shape
    p = _u(1, "p", (N, 1, H, W))
    t = _u(1, "t", (N, 1, H, W))
    s = _u(1, "s", (N, 1, H, W))
    a0 = _u(1, "a0", (N, 1, H, W))
    a1 = _u(1, "a1", (N, 1, H, W))
    d = _u(1, "d", (N, 1, 32, 32), -0.5, 1.5)
    c1, c2, c3, c4, c5, e0, e1 = 5.0, 2.5, -1.0, 2.0, 0.5, 1.5, 1.0
    g0, g1, g2 = torch.empty_like(p), torch.empty_like(p), torch.empty_like(d)
    jobs = [dict(pred=p, target=t, grad=g0, flags=GL_L1 | GL_GRAD | GL_SSIM, c_l1=c1, c_grad=c2, c_ssim=c3),
            dict(pred=p, target=t, source=s, grad=g1, flags=GL_CA, c_ca=c4, add0=a0, c_add0=e0, add1=a1, c_add1=e1),
            dict(pred=d, grad=g2, flags=GL_MSEC, c_mse=c5, t_const=1.0)]
    nj = len(jobs)
    rows = [{0: 1.0}, {1: 1.0, 2: 1.0}, {3: 1.0}, {5 + 4: 1.0}, {10 + 4: 1.0}]
    coef = [[r.get(k, 0.0) for k in range(5 * nj)] for r in rows]
    out = ops.gen_loss_fused(jobs, ([0.0] * 5, coef, [[0.0] * 4] * 5), ca=(0.15, 1.0, 3.0))

    v_l1, gl1 = ops.loss_l1(p, t)
    v_gr, ggr = ops.loss_gradient(p, t)
    v_ss, gss = ops.loss_ssim(p, t, data_range=1.0)
    v_ca, gca = ops.loss_contrast_attention(p, t, s, 0.15, 1.0, 3.0, 7)
    v_ms, gms = ops.loss_mse_const(d, 1.0)
    want = torch.stack([v_l1, v_gr, v_ss, v_ca, v_ms]).double().cpu()
    got = out.double().cpu()
    assert torch.allclose(got, want, rtol=1e-5, atol=1e-7), (got, want)
    assert _rel(g0, c1 * gl1 + c2 * ggr + c3 * gss) <= 1e-5
    assert _rel(g1, c4 * gca + e0 * a0 + e1 * a1) <= 1e-5
    assert _rel(g2, c5 * gms) <= 1e-5


def test_fused_loss_deterministic():
    from modules.hip import ops
    from modules.hip.lib import GL_GRAD, GL_L1, GL_SSIM
    p, t = _u(2, "p", (2, 1, 96, 96)), _u(2, "t", (2, 1, 96, 96))
    outs = []
    for _ in range(3):
        g = torch.empty_like(p)
        v = ops.gen_loss_fused([dict(pred=p, target=t, grad=g, flags=GL_L1 | GL_GRAD | GL_SSIM, c_l1=1.0,
                                     c_grad=1.0, c_ssim=1.0)], ([0.0], [[1.0, 1.0, 1.0, 1.0, 0.0]], [[0.0] * 4]))
        outs.append((v.clone(), g.clone()))
    for v, g in outs[1:]:
        assert torch.equal(v, outs[0][0]) and torch.equal(g, outs[0][1])
