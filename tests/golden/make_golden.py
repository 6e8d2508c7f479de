"""Generate the golden vectors in tests/golden/*.npz by running the REFERENCE itself.

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

It imports the reference's own ``modules/model.py`` (Generator, Discriminator,
ResidualBlockWithCBAM, weights layout) and ``modules/trainer.py`` (GradientLoss,
ContrastAttentionLoss, ContrastRegionLoss, ContrastEdgeLoss) with empty stand-ins
for the module-scope imports that are not installed here (torchvision,
pytorch_msssim, pydicom — an ordinary ModuleNotFoundError, not a permission
denial).  ``pytorch_msssim.SSIM`` is replaced by the oracle's restatement
(oracle/ref_torch.py::ssim), so every SSIM-dependent number is "parity unpinned".

Weights and inputs come from oracle/prng.py (splitmix64), so the fixtures hold only
inputs/outputs/gradient samples, not parameters.  Nothing from the reference is
written to disk except numerical results.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
REF = os.environ.get("DUCOSY_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from oracle import prng  # noqa: E402
from oracle import ref_torch as orc  # noqa: E402


def _install_stubs():
    tv = types.ModuleType("torchvision")
    tv.transforms = types.ModuleType("torchvision.transforms")
    tv.utils = types.ModuleType("torchvision.utils")
    tv.utils.save_image = lambda *a, **k: None
    sys.modules.update({"torchvision": tv, "torchvision.transforms": tv.transforms,
                        "torchvision.utils": tv.utils})
    pm = types.ModuleType("pytorch_msssim")

    class SSIM(torch.nn.Module):  # stand-in: oracle restatement (parity unpinned)
        def __init__(self, data_range=255, size_average=True, channel=3, **kw):
            super().__init__()
            self.data_range = data_range

        def forward(self, X, Y):
            return orc.ssim(X, Y, data_range=self.data_range)

    pm.SSIM = SSIM
    sys.modules["pytorch_msssim"] = pm
    sys.modules["pydicom"] = types.ModuleType("pydicom")


def _load_reference():
    _install_stubs()
    sys.path.insert(0, REF)
    import modules.model as rm  # noqa: E402
    import modules.trainer as rt  # noqa: E402
    return rm, rt


def _sd(shapes, seed):
    return {k: torch.from_numpy(v) for k, v in prng.init_state_dict(shapes, seed).items()}


def _grad_samples(model, tag, out):
    """Per weight: L2 norm of its gradient and 16 entries at deterministic flat indices."""
    for name, p in model.named_parameters():
        g = p.grad.detach().flatten().double().numpy()
        idx = (prng.uniform(7, "idx:" + name, (16,)) * g.size).astype(np.int64)
        out[f"{tag}gnorm:{name}"] = np.array(np.linalg.norm(g), dtype=np.float64)
        out[f"{tag}gidx:{name}"] = idx
        out[f"{tag}gval:{name}"] = g[idx].astype(np.float32)


def gen_generator(rm, cin, nb, use_cbam, n, hw, seed, fname):
    G = rm.Generator(input_channels=cin, num_residual_blocks=nb, use_cbam=use_cbam)
    shapes = {k: tuple(v.shape) for k, v in G.state_dict().items()}
    assert shapes == orc.generator_param_shapes(cin, nb, use_cbam), "layout drift"
    G.load_state_dict(_sd(shapes, seed))
    x = prng.uniform(seed, "x", (n, 1, hw, hw), -1, 1)
    if cin > 1:
        x = np.concatenate([x, prng.bernoulli(seed, "m", (n, cin - 1, hw, hw), 0.3)], 1)
    xt = torch.from_numpy(x).requires_grad_(True)
    y = G(xt)
    R = torch.from_numpy(prng.normal(seed, "R", tuple(y.shape)))
    (y * R).sum().backward()
    out = {"x": x, "y": y.detach().numpy(), "R": R.numpy(), "dx": xt.grad.numpy(),
           "meta": np.array([cin, nb, int(use_cbam), n, hw, seed])}
    _grad_samples(G, "", out)
    np.savez_compressed(os.path.join(OUT, fname), **out)


def gen_resblock(rm, n, c, hw, seed, fname):
    B = rm.ResidualBlockWithCBAM(c)
    shapes = {k: tuple(v.shape) for k, v in B.state_dict().items()}
    B.load_state_dict(_sd(shapes, seed))
    x = prng.normal(seed, "x", (n, c, hw, hw))
    xt = torch.from_numpy(x).requires_grad_(True)
    y = B(xt)
    R = torch.from_numpy(prng.normal(seed, "R", tuple(y.shape)))
    (y * R).sum().backward()
    out = {"x": x, "y": y.detach().numpy(), "R": R.numpy(), "dx": xt.grad.numpy(),
           "meta": np.array([n, c, hw, seed])}
    _grad_samples(B, "", out)
    np.savez_compressed(os.path.join(OUT, fname), **out)


def gen_discriminator(rm, n, hw, seed, fname):
    D = rm.Discriminator()
    shapes = {k: tuple(v.shape) for k, v in D.state_dict().items()}
    assert shapes == orc.discriminator_param_shapes(1)
    D.load_state_dict(_sd(shapes, seed))
    x = prng.uniform(seed, "x", (n, 1, hw, hw), -1, 1)
    xt = torch.from_numpy(x).requires_grad_(True)
    y = D(xt)
    R = torch.from_numpy(prng.normal(seed, "R", tuple(y.shape)))
    (y * R).sum().backward()
    out = {"x": x, "y": y.detach().numpy(), "R": R.numpy(), "dx": xt.grad.numpy(),
           "meta": np.array([n, hw, seed])}
    _grad_samples(D, "", out)
    np.savez_compressed(os.path.join(OUT, fname), **out)


def gen_losses(rt, n, hw, seed, fname):
    pred = np.tanh(prng.normal(seed, "pred", (n, 1, hw, hw)))
    target = prng.uniform(seed, "target", (n, 1, hw, hw), -1, 1)
    source = prng.uniform(seed, "source", (n, 1, hw, hw), -1, 1)
    crits = {
        "gradient": lambda p, t, s: rt.GradientLoss()(p, t),
        "contrast_attention": lambda p, t, s: rt.ContrastAttentionLoss(
            sigma=0.15, min_weight=1.0, max_weight=3.0, blur_kernel=7)(p, t, s),
        "contrast_region": lambda p, t, s: rt.ContrastRegionLoss(threshold=0.15, weight=1.5)(p, t, s),
        "contrast_edge": lambda p, t, s: rt.ContrastEdgeLoss()(p, t, s),
        "l1": lambda p, t, s: torch.nn.L1Loss()(p, t),
        "mse": lambda p, t, s: torch.nn.MSELoss()(p, t),
        "ssim": lambda p, t, s: sys.modules["pytorch_msssim"].SSIM(
            data_range=1.0, size_average=True, channel=1)(p, t),
    }
    out = {"pred": pred, "target": target, "source": source, "meta": np.array([n, hw, seed])}
    for name, fn in crits.items():
        p = torch.from_numpy(pred).requires_grad_(True)
        v = fn(p, torch.from_numpy(target), torch.from_numpy(source))
        v.backward()
        out[f"{name}:value"] = np.array(float(v), dtype=np.float64)
        out[f"{name}:dpred"] = p.grad.numpy()
    np.savez_compressed(os.path.join(OUT, fname), **out)


def gen_steps(rm, rt, n, hw, nb, cin, steps, seed, fname):
    """Replays modules/trainer.py:447-525 with the reference's modules/losses for `steps`
    steps of synthetic slices (real_A/real_B U(-1,1), masks Bernoulli(0.3))."""
    mk_g = lambda: rm.Generator(input_channels=cin, num_residual_blocks=nb, use_cbam=True)
    G_A2B, G_B2A, D_A, D_B = mk_g(), mk_g(), rm.Discriminator(), rm.Discriminator()
    seeds = prng.step_model_seeds(seed)
    for tag, m in (("G_A2B", G_A2B), ("G_B2A", G_B2A), ("D_A", D_A), ("D_B", D_B)):
        shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
        m.load_state_dict(_sd(shapes, seeds[tag]))
    crit_GAN, crit_cyc, crit_id = torch.nn.MSELoss(), torch.nn.L1Loss(), torch.nn.L1Loss()
    crit_grad = rt.GradientLoss()
    crit_ssim = sys.modules["pytorch_msssim"].SSIM(data_range=1.0, size_average=True, channel=1)
    crit_ca = rt.ContrastAttentionLoss(sigma=0.15, min_weight=1.0, max_weight=3.0, blur_kernel=7)
    crit_cr = rt.ContrastRegionLoss(threshold=0.15, weight=1.5)
    crit_ce = rt.ContrastEdgeLoss()
    opt_G = torch.optim.Adam(list(G_A2B.parameters()) + list(G_B2A.parameters()), lr=2e-4,
                             betas=(0.5, 0.999))
    opt_DA = torch.optim.Adam(D_A.parameters(), lr=2e-4, betas=(0.5, 0.999))
    opt_DB = torch.optim.Adam(D_B.parameters(), lr=2e-4, betas=(0.5, 0.999))
    out = {"meta": np.array([n, hw, nb, cin, steps, seed])}
    keys = ["loss_G", "loss_GAN", "loss_cycle", "loss_id", "loss_grad_cycle", "loss_grad_id",
            "loss_ssim", "loss_contrast_attention", "loss_contrast_region",
            "loss_contrast_edge", "loss_D_A", "loss_D_B"]
    hist = {k: [] for k in keys}
    for s in range(steps):
        real_A = torch.from_numpy(prng.uniform(seed, f"A{s}", (n, 1, hw, hw), -1, 1))
        real_B = torch.from_numpy(prng.uniform(seed, f"B{s}", (n, 1, hw, hw), -1, 1))
        masks = torch.from_numpy(prng.bernoulli(seed, f"M{s}", (n, cin - 1, hw, hw), 0.3))
        rA_in, rB_in = torch.cat([real_A, masks], 1), torch.cat([real_B, masks], 1)
        valid = torch.ones(n, 1, hw // 16, hw // 16)
        fake = torch.zeros(n, 1, hw // 16, hw // 16)
        # --- modules/trainer.py:463-514 ---
        opt_G.zero_grad()
        fake_B, fake_A = G_A2B(rA_in), G_B2A(rB_in)
        id_A, id_B = G_B2A(rA_in), G_A2B(rB_in)
        loss_id = (crit_id(id_A, real_A) + crit_id(id_B, real_B)) / 2
        loss_GAN = (crit_GAN(D_B(fake_B), valid) + crit_GAN(D_A(fake_A), valid)) / 2
        rec_A, rec_B = G_B2A(torch.cat([fake_B, masks], 1)), G_A2B(torch.cat([fake_A, masks], 1))
        loss_cycle = (crit_cyc(rec_A, real_A) + crit_cyc(rec_B, real_B)) / 2
        loss_grad_cycle = (crit_grad(rec_A, real_A) + crit_grad(rec_B, real_B)) / 2
        loss_grad_id = (crit_grad(id_A, real_A) + crit_grad(id_B, real_B)) / 2
        loss_ssim = 1 - ((crit_ssim(rec_A, real_A) + crit_ssim(rec_B, real_B)) / 2)
        l_ca = crit_ca(fake_B, real_B, real_A)
        l_cr = crit_cr(fake_B, real_B, real_A)
        l_ce = crit_ce(fake_B, real_B, real_A)
        loss_G = (loss_GAN + 10.0 * loss_cycle + 5.0 * loss_id + 5.0 * loss_grad_cycle
                  + 2.5 * loss_grad_id + 2.0 * loss_ssim + 2.0 * l_ca + 1.5 * l_cr + 1.0 * l_ce)
        loss_G.backward()
        opt_G.step()
        # --- modules/trainer.py:517-525 ---
        opt_DA.zero_grad()
        loss_D_A = (crit_GAN(D_A(real_A), valid) + crit_GAN(D_A(fake_A.detach()), fake)) / 2
        loss_D_A.backward()
        opt_DA.step()
        opt_DB.zero_grad()
        loss_D_B = (crit_GAN(D_B(real_B), valid) + crit_GAN(D_B(fake_B.detach()), fake)) / 2
        loss_D_B.backward()
        opt_DB.step()
        vals = [loss_G, loss_GAN, loss_cycle, loss_id, loss_grad_cycle, loss_grad_id, loss_ssim,
                l_ca, l_cr, l_ce, loss_D_A, loss_D_B]
        for k, v in zip(keys, vals):
            hist[k].append(float(v.detach()))
    for k in keys:
        out[k] = np.array(hist[k], dtype=np.float64)
    # final weights: sampled entries (weights only; pre-IN biases are noise-driven)
    for tag, m in (("G_A2B", G_A2B), ("G_B2A", G_B2A), ("D_A", D_A), ("D_B", D_B)):
        for name, p in m.named_parameters():
            if p.dim() != 4:
                continue
            w = p.detach().flatten().numpy()
            idx = (prng.uniform(11, "w:" + name, (16,)) * w.size).astype(np.int64)
            out[f"{tag}:widx:{name}"] = idx
            out[f"{tag}:wval:{name}"] = w[idx]
    np.savez_compressed(os.path.join(OUT, fname), **out)


def gen_curve(rm, rt, n, hw, nb, cin, steps, seed, threads, fname):
    """Loss curves of the reference step loop (modules/trainer.py:447-525) over `steps` steps
    at BASELINE config 1, run once per torch thread count: the spread between the runs is the
    reference's own run-to-run envelope (summation order), against which the HIP path's curve
    is judged (tests/test_gpu_curve.py).  Only the loss history is stored."""
    out = {"meta": np.array([n, hw, nb, cin, steps, seed]), "threads": np.array(threads)}
    for th in threads:
        torch.set_num_threads(th)
        tmp = os.path.join(OUT, f".curve_tmp_{th}.npz")
        gen_steps(rm, rt, n, hw, nb, cin, steps, seed, tmp)
        z = np.load(tmp)
        for k in z.files:
            if k.startswith("loss_"):
                out[f"t{th}:{k}"] = z[k]
        os.remove(tmp)
        print(f"curve: {th} threads done", flush=True)
    np.savez_compressed(os.path.join(OUT, fname), **out)


# one reference run per torch thread count: six summation orders of the same step loop
CURVE_THREADS = [1, 2, 3, 4, 6, 8]


def main():
    torch.set_num_threads(8)
    torch.manual_seed(0)
    rm, rt = _load_reference()
    if "--curve" in sys.argv:  # only the loss-curve fixture (minutes of CPU)
        gen_curve(rm, rt, 2, 128, 1, 3, 50, 601, CURVE_THREADS, "curve_128.npz")
        return
    gen_generator(rm, 3, 1, True, 2, 32, 101, "gen_cin3_nb1_32.npz")
    gen_generator(rm, 1, 9, True, 1, 32, 102, "gen_cin1_nb9_32.npz")
    gen_generator(rm, 2, 2, False, 2, 32, 103, "gen_cin2_nb2_nocbam_32.npz")
    gen_generator(rm, 3, 1, True, 1, 64, 104, "gen_cin3_nb1_64.npz")
    gen_resblock(rm, 2, 256, 16, 201, "resblock_cbam_16.npz")
    gen_discriminator(rm, 2, 64, 301, "disc_64.npz")
    gen_discriminator(rm, 1, 128, 302, "disc_128.npz")
    gen_losses(rt, 2, 64, 401, "losses_64.npz")
    gen_losses(rt, 1, 48, 402, "losses_48.npz")
    gen_steps(rm, rt, 2, 64, 1, 3, 3, 501, "steps_64.npz")
    gen_curve(rm, rt, 2, 128, 1, 3, 50, 601, CURVE_THREADS, "curve_128.npz")
    print("golden vectors written to", OUT)


if __name__ == "__main__":
    main()
