"""Per-kernel mean PMC values from a scripts/pmc_res.sh run: python scripts/pmc_table.py TAG [substring]"""
import collections
import csv
import glob
import re
import sys

tag = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "conv"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(f"gpurun_out/pmc_{tag}_*/p_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        per[(r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (did, k, c), v in per.items():
        name = re.sub(r"\(.*", "", re.sub(r"\(anonymous namespace\)::", "", k))
        agg[name[:90]][c].append(v)
for k, cs in agg.items():
    if sub not in k:
        continue
    print(k)
    print("   " + "  ".join(f"{c}={sum(v) / len(v) / 1e6:.2f}M" for c, v in sorted(cs.items())))
