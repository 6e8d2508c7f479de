"""Same convolution on two streams at once, many times: count bitwise mismatches against a
serial run.   python scripts/stress_streams.py MODE [MODE ...]"""
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "ducosy-gan_amd"); sys.path.insert(0, ".")
from oracle import prng
from test_gpu_ops import CONV_CASES, _geom, rnd
from modules.hip import ops

DEV = "cuda"
cases = [c for c in CONV_CASES if c[0] % 16 == 0 and c[1] % 16 == 0]
for mode in sys.argv[1:]:
    ops.set_mma(mode)
    sts = [torch.cuda.Stream(), torch.cuda.Stream()]
    bad = {}
    for ci, case in enumerate(cases):
        g, H = _geom(case)
        H = 64
        x = rnd((2, g.cin, H, H + 1), 41, "x").float().to(DEV).permute(0, 2, 3, 1).contiguous()
        w = torch.from_numpy(prng.normal(42, "w", (g.cout, g.cin, g.k, g.k), 0, 0.05)).float().to(DEV)
        pf, pd = g.pack_fwd(w), g.pack_dgrad(w)
        y0 = g.forward(ops.Src.nhwc(x), pf)
        d0 = g.dgrad(y0.contiguous(), pd, H, H + 1)
        torch.cuda.synchronize()
        outs = []
        for it in range(30):
            for j, st in enumerate(sts):
                st.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(st):
                    y = g.forward(ops.Src.nhwc(x), pf)
                    d = g.dgrad(y0, pd, H, H + 1)
                    outs.append((y, d))
        torch.cuda.synchronize()
        nb = sum((not torch.equal(y, y0)) + (not torch.equal(d, d0)) for y, d in outs)
        if nb:
            bad[ci] = (case, nb, max(float((y - y0).abs().max()) for y, _ in outs),
                       max(float((d - d0).abs().max()) for _, d in outs))
    print(mode, "mismatching outputs:", bad if bad else "none")
