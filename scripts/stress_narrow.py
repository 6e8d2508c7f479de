"""Stem data gradient (narrow 64->1 7x7 + reflect fold) on one stream while another stream runs
residual convs: bitwise comparison with a serial run.   python scripts/stress_narrow.py MODE"""
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from modules.hip import ops, networks as net

ops.set_mma(sys.argv[1])
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 200
MISALIGN = len(sys.argv) > 3 and sys.argv[3] == "misalign"  # non-tiled narrow kernel (no LDS halo)
DEV = "cuda"
N, H = 2, 64
L = net.gen_layers(3, 2)
stem, res, head = L["stem"], L["res"], L["head"]
dy = torch.from_numpy(prng.normal(1, "dy", (N, H, H, 64))).float().to(DEV)
if MISALIGN:
    buf = torch.empty(dy.numel() + 1, device=DEV)
    buf[1:] = dy.reshape(-1)
    dy = buf[1:].view(N, H, H, 64)
w = torch.from_numpy(prng.normal(2, "w", (64, 3, 7, 7), 0, 0.05)).float().to(DEV)
xr = torch.from_numpy(prng.normal(3, "xr", (N, H // 4, H // 4, 256))).float().to(DEV)
wr = torch.from_numpy(prng.normal(4, "wr", (256, 256, 3, 3), 0, 0.02)).float().to(DEV)
wh = torch.from_numpy(prng.normal(5, "wh", (1, 64, 7, 7), 0, 0.05)).float().to(DEV)
pr, ph = res.pack_fwd(wr), head.pack_fwd(wh)
ref = stem.dgrad(dy, stem.pack_dgrad(w, 1), H, H, ci_count=1).clone()
href = head.forward(ops.Src.nhwc(dy), ph).clone()
torch.cuda.synchronize()
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
outs, houts = [], []
for it in range(ITERS):
    s0.wait_stream(torch.cuda.current_stream())
    s1.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s1):
        for _ in range(3):
            res.forward(ops.Src.nhwc(xr), pr)
        houts.append(head.forward(ops.Src.nhwc(dy), ph))
    with torch.cuda.stream(s0):
        outs.append(stem.dgrad(dy, stem.pack_dgrad(w, 1), H, H, ci_count=1))
torch.cuda.synchronize()
bad = [i for i, o in enumerate(outs) if not torch.equal(o, ref)]
hbad = [i for i, o in enumerate(houts) if not torch.equal(o, href)]
print(sys.argv[1], ITERS, "misaligned" if MISALIGN else "aligned", "stem dgrad mismatches:", len(bad), bad[:10],
      "max", max([float((outs[i] - ref).abs().max()) for i in bad], default=0.0),
      "| head fwd mismatches:", len(hbad))
for i in bad[:4]:
    d = (outs[i] - ref).abs().squeeze(-1)  # [N, H, W]
    nz = d.nonzero()
    n_, y, x = nz[:, 0], nz[:, 1], nz[:, 2]
    print(f"  run {i}: {nz.shape[0]} elements differ; n {sorted(set(n_.tolist()))} "
          f"y {int(y.min())}..{int(y.max())} x {int(x.min())}..{int(x.max())}; "
          f"max|ref| {float(ref.abs().max()):.3g}")
