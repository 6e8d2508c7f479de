"""bench.py with ops._PHASE_F16X3 set to the given layers (comma list, "" = every phase-kernel layer on
the step's operand mode): the same-process A/B of which layers config 5's fp16 mode keeps on f16x3.
    python scripts/diag/bench_phase16.py "up1,up2,pg64,pg128,pg256" --mma f16 --no-cpu-baseline"""
import os
import runpy
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "ducosy-gan_amd"))
from modules.hip import ops  # noqa: E402

keep = sys.argv[1]
ops._PHASE_F16X3 = frozenset(x for x in keep.split(",") if x)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
