"""Does one Generator call over N images give the same parameter gradients as two calls over N/2?
(tests/test_gpu_dp_step.py at BASELINE config 4's size: the whole-batch process runs G_B2A on 48
images, a rank on 24.)  Per parameter: relative L2 of grad(N) against grad(first half) + grad(second
half), in each operand mode given (default f16x3 f32), for N in the sizes given.
    python scripts/diag/bign_split.py [N ...]  -> gpurun_out/bign_split.json"""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd")]
import torch  # noqa: E402

from oracle import prng  # noqa: E402
from oracle import ref_torch as orc  # noqa: E402

HW, NB, CIN, seed = 512, 9, 3, 921


def grads(G, x, m, dout):
    for p in G.parameters():
        p.grad = torch.zeros_like(p)
    G(x, m).backward(dout)
    return {k: p.grad.detach().clone() for k, p in G.named_parameters()}


def main():
    from modules.hip import ops
    from modules.model import Generator
    sizes = [int(v) for v in sys.argv[1:]] or [16, 48]
    sd = {k: torch.from_numpy(v) for k, v in prng.init_state_dict(orc.generator_param_shapes(CIN, NB, True), seed).items()}
    out = {}
    for mode in ("f16x3", "f32"):
        ops.set_mma(mode)
        for n in sizes:
            G = Generator(input_channels=CIN, num_residual_blocks=NB, use_cbam=True)
            G.load_state_dict(sd)
            G.cuda()
            x = torch.from_numpy(prng.uniform(seed, "A", (n, 1, HW, HW), -1, 1)).cuda()
            m = torch.from_numpy(prng.bernoulli(seed, "M", (n, CIN - 1, HW, HW), 0.3)).cuda()
            dout = torch.from_numpy(prng.normal(seed, "dout", (n, 1, HW, HW), 0, 1e-3)).cuda()
            g_all = grads(G, x, m, dout)
            h = n // 2
            g_a = grads(G, x[:h], m[:h], dout[:h])
            g_b = grads(G, x[h:], m[h:], dout[h:])
            rel = {}
            for k in g_all:
                ref = g_a[k].double() + g_b[k].double()
                if float(ref.norm()) > 0:
                    rel[k] = float((g_all[k].double() - ref).norm() / ref.norm())
            worst = sorted(rel.items(), key=lambda kv: -kv[1])[:10]
            out[f"{mode} N={n}"] = worst
            print(mode, n, worst[:6], flush=True)
            del G, g_all, g_a, g_b, x, m, dout
            torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bign_split.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
