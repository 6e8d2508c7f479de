"""Core clock during the residual weight-gradient kernel of the bench step (probe library built with
-DCLK_PROBE=1): runs bench.py's step, then reads the last launch's per-workgroup core-cycle and
wall-clock (100 MHz) counters.   DUCOSY_HIP_LIB=... python scripts/r05/clk_probe.py [bench args]"""
import ctypes
import os
import runpy
import statistics
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "ducosy-gan_amd"))


def main():
    sys.argv = [os.path.join(ROOT, "bench.py")] + (sys.argv[1:] or ["--steps", "3", "--warmup", "2", "--no-cpu-baseline"])
    try:
        runpy.run_path(sys.argv[0], run_name="__main__")
    except SystemExit:
        pass
    import torch
    from modules.hip import lib
    torch.cuda.synchronize()
    n = 4096
    buf = (ctypes.c_ulonglong * (4 * n))()
    assert lib.load().dcs_probe_clk(buf, n) == 0
    f = []
    for i in range(n):
        c0, w0, c1, w1 = buf[4 * i:4 * i + 4]
        if w1 > w0 and c1 > c0:
            f.append((c1 - c0) / ((w1 - w0) / 100e6) / 1e9)
    print(f"wgrad3 last launch: {len(f)} workgroups, core clock median {statistics.median(f):.3f} GHz "
          f"(min {min(f):.3f}, max {max(f):.3f})", flush=True)


if __name__ == "__main__":
    main()
