"""Per-layer kernel timings at the production shapes (512x512 slices, batch 8).

    python scripts/kbench.py [--batch 8] [--reps 5] [--only res]

For every convolution of the Generator / Discriminator: forward, data-gradient and
weight-gradient launch time (HIP events, median of reps) and algorithmic TFLOP/s
(2 * out_pixels * Cout * Cin * k * k per pass).  Product code only (no oracle).
"""
import argparse
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "ducosy-gan_amd"))

import torch  # noqa: E402

from modules.hip import ops  # noqa: E402
from modules.hip.lib import ACT_RELU, DCS_PAD_REFLECT, DCS_PAD_ZERO  # noqa: E402
from modules.hip.ops import ConvGeom, Src  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


LAYERS = [
    # name, geom, input H, pro (as in training, modules/hip/networks.py: the Generator's MFMA
    # convs read materialised IN outputs; the head and PatchGAN layers 1-4 apply IN + act in
    # their gather)
    ("stem", ConvGeom(3, 64, 7, 1, (3, 3, 3, 3), DCS_PAD_REFLECT), 512, False),
    ("down1", ConvGeom(64, 128, 3, 2, (1, 1, 1, 1)), 512, False),
    ("down2", ConvGeom(128, 256, 3, 2, (1, 1, 1, 1)), 256, False),
    ("res", ConvGeom(256, 256, 3, 1, (1, 1, 1, 1), DCS_PAD_REFLECT), 128, False),
    ("up1", ConvGeom(256, 128, 3, 1, (1, 1, 1, 1), DCS_PAD_ZERO, up=2), 128, False),
    ("up2", ConvGeom(128, 64, 3, 1, (1, 1, 1, 1), DCS_PAD_ZERO, up=2), 256, False),
    ("head", ConvGeom(64, 1, 7, 1, (3, 3, 3, 3), DCS_PAD_REFLECT), 512, True),
    ("d0", ConvGeom(1, 64, 4, 2, (1, 1, 1, 1)), 512, False),
    ("d1", ConvGeom(64, 128, 4, 2, (1, 1, 1, 1)), 256, True),
    ("d2", ConvGeom(128, 256, 4, 2, (1, 1, 1, 1)), 128, True),
    ("d3", ConvGeom(256, 512, 4, 2, (1, 1, 1, 1)), 64, True),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--nopro", action="store_true", help="drop the IN+ReLU gather prologue (cost probe)")
    ap.add_argument("--mma", default="f32", help="MFMA operand mode: f32 | bf16 | bf16x3 | bf16x6")
    a = ap.parse_args()
    ops.set_mma(a.mma)
    dev = torch.device("cuda")
    N = a.batch
    print(f"{'layer':8s} {'pass':6s} {'ms':>9s} {'TFLOP/s':>9s}")
    for name, g, H, pro in LAYERS:
        if a.only and name not in a.only.split(","):
            continue
        x = torch.randn(N, H, H, g.cin, device=dev)
        w = torch.randn(g.cout, g.cin, g.k, g.k, device=dev) * 0.02
        pro = pro and not a.nopro
        st = ops.in_stats(x, want_max=True) if pro else None
        pm = st.xmax if (pro and g.narrow) else None  # the head's projection kernels
        p = (st.scale, st.shift, ACT_RELU) if pro else None
        Ho, Wo = g.out_hw(H, H)
        flop = 2.0 * N * Ho * Wo * g.cout * g.cin * g.k * g.k
        if g.cin < 4:  # production layout of the stem / PatchGAN layer 0: NHWC x 4 (zero channels)
            x = torch.nn.functional.pad(x, (0, 4 - g.cin))
        wp = g.pack_fwd(w, cin_pad=x.shape[-1])
        t = timeit(lambda: g.forward(Src.nhwc(x), wp, pro=p, pro_max=pm), a.reps)
        print(f"{name:8s} {'fwd':6s} {t:9.3f} {flop / t / 1e9:9.1f}")
        sp = getattr(wp, "_dcs_sp", None)
        if sp is not None:  # the up-convs: the rows pass the sub-pixel window kernel replaces
            del wp._dcs_sp
            t = timeit(lambda: g.forward(Src.nhwc(x), wp, pro=p, pro_max=pm), a.reps)
            wp._dcs_sp = sp
            print(f"{name:8s} {'fwdrow':6s} {t:9.3f} {flop / t / 1e9:9.1f}")
        dy = torch.randn(N, Ho, Wo, g.cout, device=dev)
        wd = g.pack_dgrad(w)
        t = timeit(lambda: g.dgrad(dy, wd, H, H), a.reps)
        print(f"{name:8s} {'dgrad':6s} {t:9.3f} {flop / t / 1e9:9.1f}")
        sp = getattr(wd, "_dcs_sp", None)
        if sp is not None:  # the up-convs: the rows pass the sub-pixel window kernel replaces
            del wd._dcs_sp
            t = timeit(lambda: g.dgrad(dy, wd, H, H), a.reps)
            wd._dcs_sp = sp
            print(f"{name:8s} {'dgrow':6s} {t:9.3f} {flop / t / 1e9:9.1f}")
        t = timeit(lambda: g.wgrad(dy, Src.nhwc(x), pro=p, pro_max=pm), a.reps)
        print(f"{name:8s} {'wgrad':6s} {t:9.3f} {flop / t / 1e9:9.1f}", flush=True)
        if name == "head" and pro:  # the data gradient with the IN + ReLU backward of its input
            t = timeit(lambda: ops.in_act_backward(g.dgrad(dy, wd, H, H), x, st, ACT_RELU), a.reps)
            print(f"{name:8s} {'dg+in':6s} {t:9.3f} {'sep':>9s}")
            if ops.head_dgrad_in(dy, wd, x, st, ACT_RELU) is not None:
                t = timeit(lambda: ops.head_dgrad_in(dy, wd, x, st, ACT_RELU), a.reps)
                print(f"{name:8s} {'dg+in':6s} {t:9.3f} {'fused':>9s}", flush=True)


if __name__ == "__main__":
    main()
