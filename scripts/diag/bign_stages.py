"""Which stage of one Generator call over N images differs from the same call over the two halves?
(bign_split.py found the parameter gradients of a 48-image f16x3 call off by up to 1e-2 against two
24-image calls; f32 is exact to 3e-6.)  Per forward stage (and the input gradient): max |diff| /
max |ref| between the N-image call and the concatenated half calls, per operand mode.
    python scripts/diag/bign_stages.py [N]  -> stdout"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd")]
import torch  # noqa: E402

from oracle import prng  # noqa: E402
from oracle import ref_torch as orc  # noqa: E402

HW, NB, CIN, seed = 512, 9, 3, 921


REC = []
HEAD_WK = []


def _hook():
    """Record every backward intermediate (IN / act backward outputs, data gradients) in call order."""
    from modules.hip import ops
    def wrap(name, f):
        def g(*a, **k):
            r = f(*a, **k)
            t = r[0] if isinstance(r, tuple) else r
            if torch.is_tensor(t):
                REC.append((name, t.detach().clone()))
            return r
        return g
    for name in ("in_act_backward", "in_act_backward_parts", "cbam_backward", "act_backward"):
        setattr(ops, name, wrap(name, getattr(ops, name)))
    f_head = ops.head_dgrad_in

    def head(dy_out, wk, y, st, act):  # its inputs too
        HEAD_WK.append(wk.detach().clone())
        for k, t in (("dy_out", dy_out), ("y", y), ("scale", st.scale), ("shift", st.shift)):
            REC.append((f"head_in.{k}", t.detach().clone()))
        r = f_head(dy_out, wk, y, st, act)
        REC.append(("head_dgrad_in", r.detach().clone()))
        return r
    ops.head_dgrad_in = head
    ops.ConvGeom.dgrad = wrap("dgrad", ops.ConvGeom.dgrad)


def run(G, x, m, dout):
    from modules.hip import networks as net
    REC.clear()
    W = dict(zip(G._keys, [p for _, p in G.named_parameters()]))
    with torch.no_grad():
        out, S = net.generator_forward(W, x, m, NB, True, True)
        st = {k: S[k].clone() for k in ("y0", "a0", "y1", "a1", "y2", "h", "yu1", "au1", "yu2")}
        for k in ("s0", "s1", "s2", "su1", "su2"):
            st[k + ".scale"] = S[k].scale.clone()
        for b, blk in enumerate(S["blocks"]):
            for k in ("y1", "a1", "y2"):
                st[f"r{b}.{k}"] = getattr(blk, k).clone()
        st["out"] = out.clone()
        S["out"] = out
        dx, _ = net.generator_backward(S, dout.view(out.shape), True, 1, 0, W)
        st["dx"] = dx.clone()
        for i, (name, t) in enumerate(REC):
            st[f"bwd{i:02d}.{name}"] = t
    return st


def main():
    from modules.hip import ops
    from modules.model import Generator
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 48
    _hook()
    sd = {k: torch.from_numpy(v) for k, v in prng.init_state_dict(orc.generator_param_shapes(CIN, NB, True), seed).items()}
    for mode in ("f16x3",):
        ops.set_mma(mode)
        G = Generator(input_channels=CIN, num_residual_blocks=NB, use_cbam=True)
        G.load_state_dict(sd)
        G.cuda()
        for p in G.parameters():
            p.grad = torch.zeros_like(p)
        x = torch.from_numpy(prng.uniform(seed, "A", (n, 1, HW, HW), -1, 1)).cuda()
        m = torch.from_numpy(prng.bernoulli(seed, "M", (n, CIN - 1, HW, HW), 0.3)).cuda()
        dout = torch.from_numpy(prng.normal(seed, "dout", (n, 1, HW, HW), 0, 1e-3)).cuda()
        h = n // 2
        a = run(G, x[:h], m[:h], dout[:h])
        b = run(G, x[h:], m[h:], dout[h:])
        full = run(G, x, m, dout)
        # replay the head's fused data gradient on the recorded inputs of the N-image call, whole and in
        # halves, against the unfused path
        from modules.hip.lib import ACT_RELU, DCS_PAD_REFLECT
        from modules.hip.ops import ConvGeom, INStats
        hk = {k.split(".", 1)[1]: v for k, v in full.items() if ".head_in." in k}
        hk = {k.split(".")[-1]: v for k, v in hk.items()}
        wk = HEAD_WK[-1]
        rep = ops.head_dgrad_in(hk["dy_out"], wk, hk["y"], INStats(hk["scale"], hk["shift"]), ACT_RELU)
        halves = [ops.head_dgrad_in(hk["dy_out"][a:b].contiguous(), wk, hk["y"][a:b].contiguous(),
                                    INStats(hk["scale"][a:b].contiguous(), hk["shift"][a:b].contiguous()), ACT_RELU)
                  for a, b in ((0, h), (h, n))]
        g7 = ConvGeom(64, 1, 7, 1, (3, 3, 3, 3), DCS_PAD_REFLECT)
        unf = ops.in_act_backward(g7.dgrad(hk["dy_out"].contiguous().view(n, HW, HW, 1), wk, HW, HW), hk["y"],
                                  INStats(hk["scale"], hk["shift"]), ACT_RELU)
        ref_full = [v for k, v in full.items() if k.endswith(".head_dgrad_in")][0]
        # each half replayed on its own recorded inputs and weight pack
        for nm, rr, wkr in (("half a", a, HEAD_WK[0]), ("half b", b, HEAD_WK[1])):
            hi = {k.split(".")[-1]: v for k, v in rr.items() if ".head_in." in k}
            got = [v for k, v in rr.items() if k.endswith(".head_dgrad_in")][0]
            rp = ops.head_dgrad_in(hi["dy_out"], wkr, hi["y"], INStats(hi["scale"], hi["shift"]), ACT_RELU)
            un = ops.in_act_backward(g7.dgrad(hi["dy_out"].contiguous().view(h, HW, HW, 1), wkr, HW, HW), hi["y"],
                                     INStats(hi["scale"], hi["shift"]), ACT_RELU)
            m2 = float(un.abs().max())
            print(f"{nm}: in-step vs unfused {float((got - un).abs().max()) / m2:.3e}, replay vs unfused "
                  f"{float((rp - un).abs().max()) / m2:.3e}, wk vs full wk {float((wkr - wk).abs().max()):.3e}", flush=True)
        mx = float(unf.abs().max())
        print("replay: whole vs unfused", float((rep - unf).abs().max()) / mx, "halves vs unfused",
              float((torch.cat(halves) - unf).abs().max()) / mx, "in-step whole vs unfused",
              float((ref_full - unf).abs().max()) / mx, flush=True)
        for k, v in full.items():
            if v.shape[0] != n:
                continue
            ref = torch.cat([a[k], b[k]])
            e = float((v.double() - ref.double()).abs().max() / ref.double().abs().max().clamp_min(1e-30))
            bad = "  <--" if e > 1e-5 else ""
            print(f"{mode} N={n} {k:24s} {tuple(v.shape)} rel max {e:.3e}{bad}", flush=True)
            if bad:  # per image
                per = (v.double() - ref.double()).abs().flatten(1).max(1).values / ref.double().abs().max()
                print("   per image:", " ".join(f"{float(q):.1e}" for q in per), flush=True)


if __name__ == "__main__":
    main()
