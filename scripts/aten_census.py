"""Census of the non-library GPU launches of one bench step (ATen kernels and HIP runtime
copies / fills), grouped by the ATen operator that issued them, with input shapes.

    python scripts/aten_census.py [--img 512 --batch 8]

Runs two warm-up steps of the CycleGAN training step on synthetic data, then one step under
torch.profiler; prints per (operator, shapes) the count of device launches that are not from
libducosy_hip (kernel names not in the dcs namespace).
"""
import argparse
import collections
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ducosy-gan_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--img", type=int, default=512)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--blocks", type=int, default=9)
    a = ap.parse_args()
    from bench import _synthetic
    from modules.trainer import CycleGANSystem
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    system = CycleGANSystem(3, a.blocks, True, device=dev)
    b = _synthetic(a.batch, a.img, 2, dev, 0)
    for _ in range(2):
        system.train_step(*b)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        system.train_step(*b)
        torch.cuda.synchronize()
    # device kernels whose names are not ours, attributed to the innermost aten op
    ev = prof.events()
    cnt = collections.Counter()
    kern = collections.Counter()
    for e in ev:
        if e.device_type != torch.autograd.DeviceType.CPU:
            continue
        for k in e.kernels:
            name = k.name
            if "dcs" in name or "conv" in name.lower() and "at::" not in name:
                continue
            cnt[(e.name, str(e.input_shapes)[:90])] += 1
            kern[name[:80]] += 1
    print("== device launches by kernel")
    for k, v in kern.most_common():
        print(f"{v:5d}  {k}")
    print("== by operator (input shapes)")
    for (op, sh), v in cnt.most_common(80):
        print(f"{v:5d}  {op:40s} {sh}")
    # runtime copies / fills issued without an aten op (cudaMemcpyAsync / cudaMemsetAsync)
    rt = collections.Counter(e.name for e in ev if e.device_type == torch.autograd.DeviceType.CPU
                             and ("Memcpy" in e.name or "Memset" in e.name))
    print("== runtime API calls")
    for k, v in rt.most_common():
        print(f"{v:5d}  {k}")


if __name__ == "__main__":
    main()
