"""Platform check: a chain of deterministic PyTorch elementwise kernels on one stream (each
reads the previous kernel's output) while a second stream runs heavy unrelated work; the final
tensor is compared bit for bit with a quiet run.  No ducosy kernels on the checked stream.
   python scripts/coherence_probe.py ATTEMPTS NOISE   (NOISE: matmul | wgrad)"""
import sys
import torch
sys.path.insert(0, "ducosy-gan_amd")

attempts, noise = int(sys.argv[1]), sys.argv[2]
x0 = torch.rand(16 << 20, device="cuda")  # 64 MiB


def chain(x):
    for i in range(150):
        x = torch.sin(x * 1.0001 + 0.25)
        if i % 10 == 0:
            x = x + x.roll(12345)
    return x


ref = chain(x0.clone())
torch.cuda.synchronize()
if noise == "wgrad":
    from modules.hip import ops
    from modules.hip.lib import DCS_PAD_REFLECT
    ops.set_mma("bf16x6")
    g = ops.ConvGeom(256, 256, 3, 1, (1, 1, 1, 1), DCS_PAD_REFLECT)
    xn = torch.randn(8, 64, 64, 256, device="cuda")
A = torch.randn(4096, 4096, device="cuda")
sa, sn = torch.cuda.Stream(), torch.cuda.Stream()
bad = 0
for a in range(attempts):
    cur = torch.cuda.current_stream()
    sa.wait_stream(cur)
    sn.wait_stream(cur)
    with torch.cuda.stream(sn):
        for _ in range(60):
            if noise == "matmul":
                A = torch.tanh(A @ A * 1e-3)
            else:
                g.wgrad(xn, ops.Src.nhwc(xn))
    with torch.cuda.stream(sa):
        x = x0.clone()
        out = chain(x)
    cur.wait_stream(sa)
    cur.wait_stream(sn)
    torch.cuda.synchronize()
    if not torch.equal(out, ref):
        bad += 1
        d = (out != ref)
        print(f"  attempt {a}: {int(d.sum())} elements differ", flush=True)
print(f"noise {noise}: {bad}/{attempts} attempts differ", flush=True)
