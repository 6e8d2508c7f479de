"""Side-by-side kbench medians: python scripts/r05/kb_table.py PREFIX VARIANT... (files PREFIX{v}_{it}.log)."""
import glob
import statistics
import sys

pre, vs = sys.argv[1], sys.argv[2:]
tab = {}
for v in vs:
    for f in sorted(glob.glob(f"{pre}{v}_*.log")):
        for line in open(f):
            p = line.split()
            if len(p) >= 3 and p[0] not in ("layer",):
                try:
                    x = float(p[2])
                except ValueError:
                    continue
                tab.setdefault((p[0], p[1]), {}).setdefault(v, []).append(x)
print(f"{'layer':8s} {'pass':6s} " + " ".join(f"{v:>9s}" for v in vs))
for (l, ps), d in tab.items():
    row = [statistics.median(d[v]) if d.get(v) else float("nan") for v in vs]
    print(f"{l:8s} {ps:6s} " + " ".join(f"{x:9.3f}" for x in row))
