"""Per-instance (template arguments, workgroups) ms/step of the kernels matching a name, from
rocprofv3 kernel-trace databases:  python scripts/r05/trace_inst.py STEPS PATTERN DIR..."""
import collections
import glob
import re
import sqlite3
import sys

steps, pat = int(sys.argv[1]), sys.argv[2]
for d in sys.argv[3:]:
    agg = collections.defaultdict(lambda: [0.0, 0])
    for db in glob.glob(f"{d}/**/*.db", recursive=True):
        c = sqlite3.connect(db)
        q = ("select s.kernel_name, d.start, d.end, d.grid_size_x, d.workgroup_size_x from rocpd_kernel_dispatch d "
             "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
        for name, t0, t1, gx, wx in c.execute(q):
            if pat not in name:
                continue
            m = re.search(r"I(Li[0-9n]+E|Lb[01]E)+E", name)
            key = (m.group(0) if m else name[:40], gx // max(wx, 1))
            agg[key][0] += (t1 - t0) / 1e6 / steps
            agg[key][1] += 1
    print(d)
    for k, (ms, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"  {k[0]:34s} {k[1]:7d} WG {ms:8.3f} ms/step {n / steps:5.1f}/step {ms * steps / n * 1000:8.1f} us")
