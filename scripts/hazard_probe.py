"""Two-stream hazard probe.  Stream s1 runs bf16x6 residual convs back to
back; stream s0 runs the stem input-gradient chain: pack weights -> narrow 64->1 7x7 conv into
the padded buffer -> clone of that buffer -> reflect fold.  After one final synchronize every
tensor of every chain is compared with a single-stream reference, which separates
  (a) the narrow kernel computing a wrong buffer (the buffer itself is wrong), from
  (b) a correct buffer that the NEXT kernel on the same stream read stale (only the clone is wrong).
    python scripts/hazard_probe.py MODE KEEP N      KEEP=1: every chain's tensors stay alive
                                                    (no allocator reuse), 0: as in training"""
import ctypes
import json
import sys

import torch

sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from modules.hip import ops, networks as net, lib
from modules.hip.lib import DCS_PAD_ZERO

mode, keep, iters = sys.argv[1], sys.argv[2] == "1", int(sys.argv[3])
ops.set_mma(mode)
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
dp_ref = narrow(wp_ref).clone()
f_ref = fold(dp_ref).clone()
torch.cuda.synchronize()
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
rec = []
for it in range(iters):
    s0.wait_stream(torch.cuda.current_stream())
    s1.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s1):
        for _ in range(3):
            res.forward(ops.Src.nhwc(xr), pr)
    with torch.cuda.stream(s0):
        wp = stem.pack_dgrad(w, 1)
        dp = narrow(wp)
        dpc = dp.clone()
        f = fold(dp)
        rec.append((wp, dp, dpc, f) if keep else (wp.clone(), None, dpc, f))
torch.cuda.synchronize()
bad = []
for i, (a, b, c, d) in enumerate(rec):
    ok = (torch.equal(a, wp_ref), None if b is None else torch.equal(b, dp_ref), torch.equal(c, dp_ref),
          torch.equal(d, f_ref))
    if not all(x is not False for x in ok):
        e = {"i": i, "wp_ok": ok[0], "dp_ok": ok[1], "clone_ok": ok[2], "fold_ok": ok[3]}
        if not ok[2]:
            diff = (c != dp_ref).nonzero().tolist()
            e["clone_bad_n"] = len(diff)
            e["clone_bad_first"] = diff[:6]
            e["clone_bad_vals"] = [[float(c[tuple(x)]), float(dp_ref[tuple(x)])] for x in diff[:6]]
        bad.append(e)
print(json.dumps({"mode": mode, "keep": keep, "iters": iters, "bad": len(bad), "detail": bad[:20]}))
