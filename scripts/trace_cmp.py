"""Per-kernel ms/step of several rocprofv3 kernel-trace runs side by side:
    python scripts/trace_cmp.py STEPS DIR_A DIR_B ...   (each DIR holds one run_results.db tree)"""
import collections
import glob
import sqlite3
import sys

sys.path.insert(0, "scripts")
from hbm_table import short  # noqa: E402

steps = int(sys.argv[1])
cols = []
for d in sys.argv[2:]:
    dbs = glob.glob(f"{d}/**/*.db", recursive=True)
    agg = collections.defaultdict(float)
    for db in dbs:
        c = sqlite3.connect(db)
        for name, t0, t1 in c.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                                      "join rocpd_info_kernel_symbol s on d.kernel_id = s.id"):
            agg[short(name)] += (t1 - t0) / 1e6 / steps
    cols.append(agg)
keys = sorted(set().union(*cols), key=lambda k: -max(c.get(k, 0) for c in cols))
print(f"{'kernel':58s} " + " ".join(f"{d.rsplit('/', 1)[-1][-10:]:>10s}" for d in sys.argv[2:]))
for k in keys[:40]:
    print(f"{k[:58]:58s} " + " ".join(f"{c.get(k, 0):10.3f}" for c in cols))
print(f"{'TOTAL':58s} " + " ".join(f"{sum(c.values()):10.3f}" for c in cols))
