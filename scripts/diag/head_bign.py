"""ops.head_dgrad_in (the head's data gradient fused with the IN + ReLU backward of its input,
csrc/conv_head.hip) at N images against the same call split into pieces, and against the unfused
path (head dgrad, then in_act_backward).  bign_stages.py found its output off by up to 0.36 at N = 48
against two 24-image calls.
    python scripts/diag/head_bign.py [N ...]"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd")]
import torch  # noqa: E402


def main():
    from modules.hip import ops
    from modules.hip.lib import ACT_RELU, DCS_PAD_REFLECT
    from modules.hip.ops import ConvGeom
    ops.set_mma("f16x3")
    H = 512
    g = ConvGeom(64, 1, 7, 1, (3, 3, 3, 3), DCS_PAD_REFLECT)
    torch.manual_seed(0)
    w = torch.randn(1, 64, 7, 7, device="cuda") * 0.02
    wk = g.pack_dgrad(w)
    for n in [int(v) for v in sys.argv[1:]] or [8, 24, 32, 33, 48]:
        y = torch.randn(n, H, H, 64, device="cuda")
        st = ops.in_stats(y, want_max=True)
        dout = torch.randn(n, 1, H, H, device="cuda") * 1e-3
        full = ops.head_dgrad_in(dout, wk, y, st, ACT_RELU)
        ref = ops.in_act_backward(g.dgrad(dout.view(n, H, H, 1), wk, H, H), y, st, ACT_RELU)
        e_ref = (full - ref).abs().flatten(1).max(1).values / ref.abs().max()
        pieces = []
        for a in range(0, n, 8):
            b = min(n, a + 8)
            st_p = ops.INStats(st.scale[a:b].contiguous(), st.shift[a:b].contiguous(), st.xmax[a:b].contiguous(), None)
            pieces.append(ops.head_dgrad_in(dout[a:b].contiguous(), wk, y[a:b].contiguous(), st_p, ACT_RELU))
        e_pc = (full - torch.cat(pieces)).abs().flatten(1).max(1).values / ref.abs().max()
        print(f"N={n}: fused vs unfused max {float(e_ref.max()):.2e}, worst images {e_ref.topk(min(4, n)).indices.tolist()}; "
              f"vs 8-image pieces max {float(e_pc.max()):.2e}", flush=True)
        del y, st, dout, full, ref, pieces
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
