"""Input-pipeline throughput on one GPU: HU transform + anatomical masks for one training batch
(8 NCCT slices 512x512 -> soft-tissue masks ['bone', 'mediastinum'] or all four kinds), timed
with HIP events on the launch stream; the CPU restatement (oracle/masks_ref.py, the reference
algorithm with scipy/numpy) timed beside it on a few slices.

    python scripts/bench_masks.py [--batch 8] [--size 512] [--iters 20] [--kinds bone,mediastinum]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ducosy-gan_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from modules import phantom  # noqa: E402
from modules.hip import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--kinds", default="bone,mediastinum")
    ap.add_argument("--cpu-slices", type=int, default=3)
    a = ap.parse_args()
    kinds = a.kinds.split(",")
    dev = torch.device("cuda:0")
    raw, slope, inter = phantom.ct_batch(7, a.batch, a.size, kinds=("chest",))
    r, s, i = (torch.from_numpy(x).to(dev) for x in (raw, slope, inter))
    out = torch.empty(a.batch, len(kinds), a.size, a.size, device=dev)

    def step():
        hu, img = ops.hu_transform(r, s, i, -150, 250, soft=True)
        ops.anatomical_masks(hu, kinds, out=out)
        return img

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(a.iters):
        step()
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / a.iters

    sys.path.insert(0, ROOT)
    from oracle import masks_ref
    t0 = time.perf_counter()
    for n in range(a.cpu_slices):
        hu, img = masks_ref.hu_transform(raw[n], slope[n], inter[n], -150, 250, True)
        masks_ref.masks_2d(hu, kinds)
    cpu = (time.perf_counter() - t0) / a.cpu_slices
    px = a.batch * a.size * a.size
    print(json.dumps({"workload": f"HU transform + masks {kinds}, {a.batch}x{a.size}^2 int16 slices",
                      "ms_per_batch": round(ms, 4), "slices_per_s": round(a.batch / ms * 1e3, 1),
                      "mpix_per_s": round(px / ms / 1e3, 1),
                      "cpu_oracle_ms_per_slice": round(cpu * 1e3, 2), "cpu_threads": 1}))


if __name__ == "__main__":
    main()
