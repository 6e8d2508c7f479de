"""Which of the stem data gradient's three kernels (weight pack, narrow 64->1 7x7 conv into
the padded buffer, reflect fold) goes wrong while another stream runs bf16-mode residual
convs?   python scripts/stress_narrow2.py MODE"""
import ctypes
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from modules.hip import ops, networks as net, lib
from modules.hip.lib import DCS_PAD_ZERO

ops.set_mma(sys.argv[1])
DEV = "cuda"
N, H, p = 2, 64, 3
L = net.gen_layers(3, 2)
stem, res = L["stem"], L["res"]
dy = torch.from_numpy(prng.normal(1, "dy", (N, H, H, 64))).float().to(DEV)
w = torch.from_numpy(prng.normal(2, "w", (64, 3, 7, 7), 0, 0.05)).float().to(DEV)
xr = torch.from_numpy(prng.normal(3, "xr", (N, H // 4, H // 4, 256))).float().to(DEV)
wr = torch.from_numpy(prng.normal(4, "wr", (256, 256, 3, 3), 0, 0.02)).float().to(DEV)
pr = res.pack_fwd(wr)


def narrow(wp):
    d = lib.ConvDesc()
    d.N, d.Hs, d.Ws, d.Cs = N, H, H, 64
    d.s_n, d.s_c, d.s_h, d.s_w = H * H * 64, 1, H * 64, 64
    d.csplit, d.up, d.pad_mode, d.KH, d.KW = 64, 1, DCS_PAD_ZERO, 7, 7
    d.ldb, d.mma, d.Co, d.stride, d.parity, d.pt, d.pl = wp.shape[1], 0, 1, 1, 0, 6, 6
    d.Ho, d.Wo = H + 2 * p, H + 2 * p
    out = torch.empty(N, d.Ho, d.Wo, 1, device=DEV)
    lib.call("dcs_conv_rows_narrow", ctypes.byref(d), ops._p(dy), None, ops._p(wp), None, None, None,
             ops._p(out), ops._stream())
    return out


def fold(dpad):
    out = torch.empty(N, H, H, 1, device=DEV)
    lib.call("dcs_reflect_fold", ops._p(dpad), None, ops._p(out), N, H, H, 1, p, ops._stream())
    return out


wp_ref = stem.pack_dgrad(w, 1).clone()
dpad_ref = narrow(wp_ref).clone()
out_ref = fold(dpad_ref).clone()
torch.cuda.synchronize()
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
rec = {"pack": [], "narrow": [], "fold": []}
CHAIN = len(sys.argv) > 2 and sys.argv[2] == "chain"  # pack -> narrow -> clone(dpad) -> fold, one stream
chain = []
for it in range(int(sys.argv[3]) if len(sys.argv) > 3 else 300):
    s0.wait_stream(torch.cuda.current_stream())
    s1.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s1):
        for _ in range(3):
            res.forward(ops.Src.nhwc(xr), pr)
    with torch.cuda.stream(s0):
        k = it % 3
        if CHAIN:
            wp = stem.pack_dgrad(w, 1)
            dp = narrow(wp)
            chain.append((wp.clone(), dp.clone(), fold(dp)))
            continue
        if k == 0:
            rec["pack"].append(stem.pack_dgrad(w, 1))
        elif k == 1:
            rec["narrow"].append(narrow(wp_ref))
        else:
            rec["fold"].append(fold(dpad_ref))
torch.cuda.synchronize()
if CHAIN:
    bad = [(i, torch.equal(a, wp_ref), torch.equal(b, dpad_ref), torch.equal(c, out_ref))
           for i, (a, b, c) in enumerate(chain)
           if not (torch.equal(a, wp_ref) and torch.equal(b, dpad_ref) and torch.equal(c, out_ref))]
    print(sys.argv[1], "chain", len(chain), "mismatching chains (i, pack ok, dpad clone ok, fold ok):", bad[:12])
    sys.exit(0)
refs = {"pack": wp_ref, "narrow": dpad_ref, "fold": out_ref}
for k, v in rec.items():
    bad = [i for i, o in enumerate(v) if not torch.equal(o, refs[k])]
    print(sys.argv[1], k, f"{len(bad)}/{len(v)} mismatching", [int((v[i] != refs[k]).sum()) for i in bad[:8]])
