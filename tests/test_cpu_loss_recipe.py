"""Host logic of the fused G-step loss: the coefficient recipe that composes the reported loss
terms and loss_G from the fused kernel's per-job term means (modules/trainer.py
CycleGANSystem._g_loss_recipe) equals the reference's composition (trainer.py:469-512)."""
import random
import types

import pytest


def test_g_loss_recipe_matches_reference_composition():
    from modules import trainer
    lc, li = 10.0, 5.0
    me = types.SimpleNamespace(lambda_cyc=lc, lambda_id=li)
    bias, coef, coefx = trainer.CycleGANSystem._g_loss_recipe(me, 7)
    rnd = random.Random(3)
    v = [rnd.uniform(0.0, 1.0) for _ in range(35)]  # val[5 j + q]
    cr, ce = rnd.uniform(0, 1), rnd.uniform(0, 1)
    out = {k: bias[i] + sum(c * x for c, x in zip(coef[i], v)) + coefx[i][0] * cr + coefx[i][1] * ce
           for i, k in enumerate(trainer._G_TERMS)}
    V = lambda j, q: v[5 * j + q]  # noqa: E731  jobs: 0 rec_A, 1 rec_B, 2 id_A, 3 id_B, 4 fake_B, 5/6 D outputs
    grad = lambda j: V(j, 1) + V(j, 2)  # noqa: E731  GradientLoss = x-part mean + y-part mean
    want = {
        "loss_GAN": (V(5, 4) + V(6, 4)) / 2,
        "loss_cycle": (V(0, 0) + V(1, 0)) / 2,
        "loss_id": (V(2, 0) + V(3, 0)) / 2,
        "loss_grad_cycle": (grad(0) + grad(1)) / 2,
        "loss_grad_id": (grad(2) + grad(3)) / 2,
        "loss_ssim": 1 - (V(0, 3) + V(1, 3)) / 2,
        "loss_contrast_attention": V(4, 4),
        "loss_contrast_region": cr,
        "loss_contrast_edge": ce,
    }
    want["loss_G"] = (want["loss_GAN"] + lc * want["loss_cycle"] + li * want["loss_id"]
                      + trainer.LAMBDA_GRAD * want["loss_grad_cycle"] + trainer.LAMBDA_GRAD_ID * want["loss_grad_id"]
                      + trainer.LAMBDA_SSIM * want["loss_ssim"] + trainer.LAMBDA_CA * want["loss_contrast_attention"]
                      + trainer.LAMBDA_CR * want["loss_contrast_region"] + trainer.LAMBDA_CE * want["loss_contrast_edge"])
    for k in trainer._G_TERMS:
        assert out[k] == pytest.approx(want[k], rel=1e-12, abs=1e-12), k


def test_reference_lambdas():
    """trainer.py:493-502 weights."""
    from modules import trainer
    assert (trainer.LAMBDA_GRAD, trainer.LAMBDA_GRAD_ID, trainer.LAMBDA_SSIM) == (5.0, 2.5, 2.0)
    assert (trainer.LAMBDA_CA, trainer.LAMBDA_CR, trainer.LAMBDA_CE) == (2.0, 1.5, 1.0)
