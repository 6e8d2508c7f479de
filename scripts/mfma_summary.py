"""MFMA-busy fraction of the residual conv kernel from a scripts/pmc_mfma.sh pass.

    python scripts/mfma_summary.py TAG MODE [MODE ...]     -> profiles/TAG_mfma_busy.json

Per dispatch: SQ_VALU_MFMA_BUSY_CYCLES is summed over all 1024 SIMDs (= cycles per MFMA x
MFMAs); GRBM_GUI_ACTIVE is summed over the 8 XCDs.  busy = MFMA_BUSY / (1024 * GUI_ACTIVE/8).
The dispatch's own timestamps give its duration and the implied shader clock.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
TAGS = {"f32": 0, "bf16": 1, "bf16x3": 3, "bf16x6": 6}


def summarise(tag, mode):
    path = glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{tag}_mfma_{mode}", "**", "p_counter_collection.csv"),
                     recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(path)):
        k = r["Dispatch_Id"]
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[k] = (r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    name = f"conv_rows_kernel<128, 128, 1, 1, {TAGS[mode]}>"
    ks = [k for k in per if name in meta[k][0]]
    busy = [per[k]["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * per[k]["GRBM_GUI_ACTIVE"] / 8) for k in ks]
    dur = [(meta[k][2] - meta[k][1]) * 1e-9 for k in ks]
    clk = [per[k]["GRBM_GUI_ACTIVE"] / 8 / d / 1e9 for k, d in zip(ks, dur)]
    return {"kernel": name, "dispatches": len(ks), "mfma_busy_fraction": round(sum(busy) / len(busy), 4),
            "mean_duration_ms": round(sum(dur) / len(dur) * 1e3, 4), "implied_clock_ghz": round(sum(clk) / len(clk), 3),
            "mfma_instructions_per_dispatch": round(sum(per[k]["SQ_INSTS_MFMA"] for k in ks) / len(ks))}


if __name__ == "__main__":
    tag, modes = sys.argv[1], sys.argv[2:] or ["f32"]
    try:  # merge: modes profiled in earlier passes stay
        out = json.load(open(os.path.join(ROOT, "profiles", "mfma_busy.json")))
    except (OSError, ValueError):
        out = {}
    out.update({m: summarise(tag, m) for m in modes})
    out["source"] = (f"rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- "
                     f"bench.py --steps 1 --warmup 1 --mma MODE (scripts/pmc_mfma.sh, tag {tag})")
    for fn in (f"{tag}_mfma_busy.json", "mfma_busy.json"):  # tagged record + the copy bench.py reads
        with open(os.path.join(ROOT, "profiles", fn), "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
