"""Fixed (per-workgroup prologue / epilogue) cost of the residual window conv: forward launch time
at N=16, 128x128, Cout 256 for Cin 64 .. 512; a line T = a + b * Cin fitted through the points gives
a, the part of a launch that does not scale with the k loop.
    python scripts/r05/fixed_cost.py [--mma f16x3]"""
import argparse
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "ducosy-gan_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

from kbench import timeit  # noqa: E402
from modules.hip import ops  # noqa: E402
from modules.hip.lib import DCS_PAD_REFLECT  # noqa: E402
from modules.hip.ops import ConvGeom, Src  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mma", default="f16x3")
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    ops.set_mma(a.mma)
    N, H, Co = a.batch, 128, 256
    pts = []
    for cin in (64, 128, 256, 512):
        g = ConvGeom(cin, Co, 3, 1, (1, 1, 1, 1), DCS_PAD_REFLECT)
        x = torch.randn(N, H, H, cin, device="cuda")
        w = torch.randn(Co, cin, 3, 3, device="cuda") * 0.02
        wp = g.pack_fwd(w, cin_pad=cin)
        t = timeit(lambda: g.forward(Src.nhwc(x), wp), 9)
        dy = torch.randn(N, H, H, Co, device="cuda")
        tw = timeit(lambda: g.wgrad(dy, Src.nhwc(x)), 9)
        pts.append((cin, t, tw))
        print(f"cin {cin:4d}  fwd {t * 1e3:8.1f} us  wgrad {tw * 1e3:8.1f} us", flush=True)
    for k, name in ((1, "fwd"), (2, "wgrad")):
        xs = [p[0] for p in pts]
        ys = [p[k] * 1e3 for p in pts]
        n = len(xs)
        mx, my = sum(xs) / n, sum(ys) / n
        b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
        print(f"{name}: T = {my - b * mx:.1f} us + {b:.3f} us * Cin  (Cin 256: fixed share "
              f"{(my - b * mx) / (my - b * mx + 256 * b):.3f})")


if __name__ == "__main__":
    main()
