"""Outputs of the residual conv passes for seeded inputs, saved for a bit-exactness comparison
between two library builds (run once per build with DUCOSY_HIP_LIB set):

    python scripts/lib_outputs.py OUT.pt        then      python scripts/lib_outputs.py --cmp A.pt B.pt
"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "ducosy-gan_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    if sys.argv[1] == "--cmp":
        a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
        bad = [k for k in a if not torch.equal(a[k], b[k])]
        for k in bad:
            print("DIFF", k, float((a[k] - b[k]).abs().max()))
        print("identical" if not bad else f"{len(bad)} of {len(a)} differ", len(a))
        sys.exit(1 if bad else 0)
    from oracle import prng
    from modules.hip import ops
    from modules.hip.lib import DCS_PAD_REFLECT
    ops.set_mma("bf16x6")
    g = ops.ConvGeom(256, 256, 3, 1, (1, 1, 1, 1), DCS_PAD_REFLECT)
    out = {}
    for n, h in ((1, 16), (3, 32), (16, 128), (2, 24)):
        x = torch.from_numpy(prng.normal(81, f"x{n}{h}", (n, h, h, 256))).float().cuda()
        w = torch.from_numpy(prng.normal(82, "w", (256, 256, 3, 3), 0, 0.02)).float().cuda()
        dy = torch.from_numpy(prng.normal(83, f"dy{n}{h}", (n, h, h, 256))).float().cuda()
        wp = g.pack_fwd(w)
        out[f"fwd{n}_{h}"] = g.forward(ops.Src.nhwc(x), wp).cpu()
        y, st = g.forward_in_stats(ops.Src.nhwc(x), wp)
        out[f"fwds{n}_{h}"] = y.cpu()
        out[f"scale{n}_{h}"] = st.scale.cpu()
        out[f"shift{n}_{h}"] = st.shift.cpu()
        out[f"dgrad{n}_{h}"] = g.dgrad(dy, g.pack_dgrad(w), h, h).cpu()
        out[f"wgrad{n}_{h}"] = g.wgrad(dy, ops.Src.nhwc(x)).cpu()
    torch.save(out, sys.argv[1])
    print("saved", len(out))


if __name__ == "__main__":
    main()
