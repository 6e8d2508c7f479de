"""Determinism of the window conv forward / data gradient (batch of 3 at 128 x 128 x 256) across repeated
launches and against per-image launches: prints max |difference| per comparison.
    DUCOSY_HIP_LIB=... python scripts/diag/win_async_check.py"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "ducosy-gan_amd")]
import torch  # noqa: E402
from oracle import prng  # noqa: E402
from modules.hip import ops  # noqa: E402
from test_gpu_win import _geom, rnd  # noqa: E402

ops.set_mma("f16x3")
g = _geom(ops)
N, H, W = 3, 128, 128
xd = rnd((N, 256, H, W), 71, "x").float().cuda().permute(0, 2, 3, 1).contiguous()
w = torch.from_numpy(prng.normal(72, "w", (256, 256, 3, 3), 0, 0.05)).float().cuda()
wp = g.pack_fwd(w)
ys = [g.forward_in_stats(ops.Src.nhwc(xd), wp, want_max=True)[0].clone() for _ in range(4)]
print("repeat max|d|:", [float((y - ys[0]).abs().max()) for y in ys[1:]])
for i in range(N):
    yi = g.forward_in_stats(ops.Src.nhwc(xd[i:i + 1].contiguous()), wp, want_max=True)[0]
    d = (ys[0][i:i + 1] - yi).abs()
    print(f"image {i}: max|d| {float(d.max()):.3e}, pixels differing {int((d.amax(dim=3) > 0).sum())}")
    if float(d.max()) > 0:
        idx = (d.amax(dim=3)[0] > 0).nonzero()[:8].tolist()
        print("   first differing (row, col):", idx)
print("range exps:", ops.range_rec(xd).max().item(), [ops.range_rec(xd[i:i+1].contiguous()).max().item() for i in range(N)])
