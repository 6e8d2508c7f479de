"""Per-workgroup phase times of the residual window conv forward (probe library built with
-DWIN_TIMING=1: DUCOSY_HIP_LIB=.../libducosy_hip_tm.so): prologue (start -> first barrier), k loop,
epilogue (stores retired), and the gap between a CU's consecutive workgroups.
    python scripts/r05/win_timing.py [--batch 16] [--cin 256]"""
import argparse
import collections
import ctypes
import os
import statistics
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "ducosy-gan_amd"))

import torch  # noqa: E402

from modules.hip import lib, ops  # noqa: E402
from modules.hip.lib import DCS_PAD_REFLECT  # noqa: E402
from modules.hip.ops import ConvGeom, Src  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--cin", type=int, default=256)
    a = ap.parse_args()
    ops.set_mma("f16x3")
    N, H, Co, cin = a.batch, 128, 256, a.cin
    g = ConvGeom(cin, Co, 3, 1, (1, 1, 1, 1), DCS_PAD_REFLECT)
    x = torch.randn(N, H, H, cin, device="cuda")
    w = torch.randn(Co, cin, 3, 3, device="cuda") * 0.02
    wp = g.pack_fwd(w, cin_pad=cin)
    for _ in range(3):
        g.forward(Src.nhwc(x), wp)
    torch.cuda.synchronize()
    nwg = N * (H * H // 256) * (Co // 128)
    buf = (ctypes.c_ulonglong * (5 * nwg))()
    assert lib.load().dcs_probe_win_times(buf, nwg) == 0
    rec = [tuple(buf[5 * i:5 * i + 5]) for i in range(nwg)]
    t00 = min(r[0] for r in rec)
    us = 0.01  # s_memrealtime: 100 MHz
    pro = [(r[1] - r[0]) * us for r in rec]
    loop = [(r[2] - r[1]) * us for r in rec]
    epi = [(r[3] - r[2]) * us for r in rec]
    span = (max(r[3] for r in rec) - t00) * us
    bycu = collections.defaultdict(list)
    for r in rec:
        bycu[r[4]].append(r)
    gaps, firsts = [], []
    for cu, rs in bycu.items():
        rs.sort()
        firsts.append((rs[0][0] - t00) * us)
        for p, q in zip(rs, rs[1:]):
            gaps.append((q[0] - p[3]) * us)
    med = statistics.median
    print(f"workgroups {nwg}  CUs {len(bycu)}  span {span:.1f} us  (WG/CU {nwg / len(bycu):.1f})")
    print(f"prologue  median {med(pro):6.2f} us  max {max(pro):6.2f}")
    print(f"k loop    median {med(loop):6.2f} us  max {max(loop):6.2f}  min {min(loop):6.2f}")
    print(f"epilogue  median {med(epi):6.2f} us  max {max(epi):6.2f}")
    print(f"gap       median {med(gaps):6.2f} us  max {max(gaps):6.2f}  (end of a WG -> start of the next on its CU)")
    print(f"first start: median {med(firsts):6.2f} us  max {max(firsts):6.2f}")
    tot = sum(pro) + sum(loop) + sum(epi) + sum(gaps)
    print(f"shares: prologue {sum(pro) / tot:.3f}  loop {sum(loop) / tot:.3f}  epilogue {sum(epi) / tot:.3f}  "
          f"gap {sum(gaps) / tot:.3f}")


if __name__ == "__main__":
    main()
