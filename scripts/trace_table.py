"""Per-kernel time table from a rocprofv3 --kernel-trace database (run_results.db).

    python scripts/trace_table.py DB [STEPS]   (STEPS: timed + warm-up steps of the traced bench run,
                                                 used to print ms per step; default 7 = 5 + 2)
"""
import collections
import sqlite3
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from hbm_table import short  # noqa: E402


def main(db, steps=7):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
        "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
    agg = collections.defaultdict(list)
    for name, t0, t1 in rows:
        agg[short(name)].append((t1 - t0) / 1e3)
    tot = sum(sum(v) for v in agg.values())
    print(f"{'kernel':60s} {'calls':>6s} {'ms/step':>8s} {'avg us':>8s}")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k[:60]:60s} {len(v) / steps:6.1f} {sum(v) / 1e3 / steps:8.2f} {sum(v) / len(v):8.1f}")
    print(f"total kernel ms/step {tot / 1e3 / steps:.2f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 7)
