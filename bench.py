"""Benchmark: CycleGAN train-step images/sec at 512x512, bs=8 per GPU (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step is one full pass of modules/trainer.py:463-525 (G step with all nine loss terms and
its Adam, D_A step, D_B step) on the fused HIP path, over one synthetic batch of 8 slices per
GPU that is already resident in HBM.  Data parallel: one process per GPU, each with its own
shard; one RCCL all-reduce per optimizer (weak scaling).  Rank 0 prints ONE JSON line.

MFMA operand mode (--mma): f16x3 by default, an fp32-class split (each fp32 operand, scaled by a
power of two from its range record, = hi + lo fp16; three fp16 MFMAs per product, fp32
accumulation and storage; its measured error against float64 is at or below the exact-f32 MFMA
path's on every layer, tests/test_gpu_mma.py); --mma f32 runs the exact v_mfma_f32_32x32x2_f32
path; --mma f16 is BASELINE config 5's fp16 MFMA path (one product of the scaled fp16 operands).

roofline: the dominant kernel is the 256-ch 3x3 residual-block convolution (forward + data-gradient
launches; in the fp16 modes the 16x16x32 window kernel conv3_win16_kernel).  Its per-launch duration is
measured live with HIP events on the launch stream over the timed steps; FLOPs are algorithmic
(2*pixels*256*256*9 per launch).  Peak: 157.3 TFLOP/s for f32 (gfx950 f32 MFMA, dense); the dense
fp16/bf16 MFMA peak (2.5 PF) divided by the products per fragment pair in the split modes (f16x3:
3 -> 838.9 TFLOP/s of fp32 work; bf16x6: 6 -> 419.5).
cpu_baseline: the oracle (oracle/ref_torch.py, the CPU restatement of the reference step)
timed on this host on a bounded sample (one 512x512 slice, 9 blocks, one step).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ducosy-gan_amd"))

import torch  # noqa: E402

F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, dense
BF16_MFMA_PEAK_TFLOPS = 16 * F32_MFMA_PEAK_TFLOPS  # v_mfma_f32_32x32x16_bf16: 16x the f32 rate (~2.5 PF dense)
# peak per mode for the dominant kernel's algorithmic FLOPs: bf16x3 issues 3 bf16 MFMAs per product
MODE_PEAK = {"f32": F32_MFMA_PEAK_TFLOPS, "bf16": BF16_MFMA_PEAK_TFLOPS, "bf16x3": BF16_MFMA_PEAK_TFLOPS / 3,
             "bf16x6": BF16_MFMA_PEAK_TFLOPS / 6, "f16x3": BF16_MFMA_PEAK_TFLOPS / 3, "f16": BF16_MFMA_PEAK_TFLOPS}
MODE_DTYPE = {"f32": "f32", "bf16": "bf16 (MFMA operands; f32 accumulation and storage)",
              "bf16x3": "f32 via bf16x3 MFMA (hi/lo split, ~2^-16 per product; f32 accumulation and storage)",
              "bf16x6": "f32 via bf16x6 MFMA (hi/mid/lo split, ~2^-24 per product; f32 accumulation and storage)",
              "f16x3": "f32 via f16x3 MFMA (power-of-two scaled hi/lo fp16 split, 22 significant bits, three "
                       "products; f32 accumulation and storage)",
              "f16": "f16 (MFMA operands: power-of-two scaled fp16, one product; f32 accumulation and storage)"}
MODE_TAG = {"f32": 0, "bf16": 1, "bf16x3": 3, "bf16x6": 6, "f16x3": 7, "f16": 8}
HBM_PEAK_GBS = 8000.0


def _synthetic(n, img, n_masks, device, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    a = torch.rand(n, 1, img, img, generator=g, device=device) * 2 - 1
    b = torch.rand(n, 1, img, img, generator=g, device=device) * 2 - 1
    m = (torch.rand(n, n_masks, img, img, generator=g, device=device) < 0.3).float() if n_masks else None
    return a, b, m


def _cpu_steps(img, bs, blocks, cin, warmup, steps):
    """Median seconds per step of the oracle's CPU train step (the reference algorithm restated,
    oracle/ref_torch.py, fp32) after ``warmup`` untimed steps."""
    from oracle import prng
    from oracle import ref_torch as orc
    gs, ds = orc.generator_param_shapes(cin, blocks, True), orc.discriminator_param_shapes(1)
    sd = lambda shapes, s: {k: torch.from_numpy(v) for k, v in prng.init_state_dict(shapes, s).items()}
    m = orc.OracleCycleGAN(sd(gs, 1), sd(gs, 2), sd(ds, 3), sd(ds, 4), blocks)
    a = torch.from_numpy(prng.uniform(5, "A", (bs, 1, img, img), -1, 1))
    b = torch.from_numpy(prng.uniform(5, "B", (bs, 1, img, img), -1, 1))
    mk = torch.from_numpy(prng.bernoulli(5, "M", (bs, cin - 1, img, img), 0.3)) if cin > 1 else None
    for _ in range(warmup):  # first-call oneDNN primitive setup stays out of the timing
        m.step(a, b, mk)
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        m.step(a, b, mk)
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def cpu_baseline(img, blocks, cin, threads):
    """BASELINE.md section 3 on this host's cores: the oracle's CPU step at BASELINE config 1 (128x128,
    bs 2, 1 residual block) and at the metric's shape (512x512, bs 1, 9 blocks), 3 untimed warm-up
    steps each, median of the timed steps.  ``value`` is the 512x512 rate (same slice shape as the
    GPU metric); the 512x512 sample is 3 timed steps to keep the default bench within minutes."""
    sys.path.insert(0, ROOT)
    torch.set_num_threads(threads)
    c1 = _cpu_steps(128, 2, 1, cin, 3, 10)
    full = _cpu_steps(img, 1, blocks, cin, 3, 3)
    cpu = "?"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(1.0 / full, 4), "unit": "img/s", "cores": threads, "kind": "port", "cpu": cpu,
            "config1_img_s": round(2.0 / c1, 3),
            "sample": f"oracle/ref_torch.py fp32 CPU train step (G+D_A+D_B, all losses, Adam), median after 3 "
                      f"untimed warm-ups: {img}x{img} bs 1, {blocks} blocks, cin {cin}, 3 timed steps "
                      f"({full:.2f} s/step) = value; BASELINE config 1 (128x128 bs 2, 1 block) 10 timed steps "
                      f"({c1 * 1e3:.0f} ms/step) = config1_img_s"}


def all_finite(tensors) -> bool:
    """One device-side verdict over every tensor: True when none holds a NaN or an infinity.  A step
    whose numbers went bad must not be reported (round 5: a kernel that wrote NaN ran faster, since NaN
    operands draw less power)."""
    flags = [torch.isfinite(t.detach()).all().reshape(1) for t in tensors if t.numel()]
    return bool(torch.cat(flags).all().item()) if flags else True


def _pmc_record(mode):
    """HBM bytes per launch (2*FETCH_SIZE + WRITE_SIZE, gfx950 FETCH correction) and MFMA-busy of the
    dominant kernel from the committed rocprofv3 PMC passes (profiles/pmc_resconv_MODE.json, written
    by scripts/hbm_table.py).  PMC passes cannot run inside the timed loop, so these are NOT
    measured in this run: the record carries the profile's commit and source next to them."""
    p = os.path.join(ROOT, "profiles", f"pmc_resconv_{mode}.json")
    try:
        with open(p) as f:
            j = json.load(f)
    except (OSError, ValueError):
        return None, None, None
    src = f"{j.get('source', p)} at commit {j.get('commit', '?')}"
    return j.get("hbm_bytes_per_launch"), j.get("mfma_busy_fraction"), src


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="per-GPU batch")
    ap.add_argument("--img", type=int, default=512)
    ap.add_argument("--blocks", type=int, default=9)
    ap.add_argument("--cin", type=int, default=3, help="1 + masks (soft tissue: 3, lung: 2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mma", default="f16x3", choices=["f32", "bf16", "bf16x3", "bf16x6", "f16x3", "f16"],
                    help="MFMA operand mode of the conv passes: f16x3 = power-of-two scaled hi/lo fp16 split, "
                         "three products, fp32-class (default; error <= the exact-f32 path's, "
                         "tests/test_gpu_mma.py), bf16x6 = three-way bf16 split (fp32-class, 6 products), "
                         "f32 = exact fp32 MFMA, bf16x3 = hi/lo bf16 split, bf16 = plain bf16 operands, "
                         "f16 = scaled fp16 operands, one product (BASELINE config 5's fp16 MFMA path)")
    ap.add_argument("--dual", action="store_true",
                    help="BASELINE config 5: soft-tissue (cin 3) and lung (cin 2) CycleGANs trained in one "
                         "process; value counts the images of both models")
    ap.add_argument("--dual-schedule", default="serial", choices=["serial", "groups"],
                    help="--dual: both models one after the other on each GPU (serial; trainer.py "
                         "ConcurrentCycleGANs), or split GPU groups (groups: soft tissue on the first half of the "
                         "ranks, lung on the second, each with its own all-reduce)")
    ap.add_argument("--inject-nan", action="store_true",
                    help="test hook: put a NaN into the synthetic inputs (the run must then exit non-zero)")
    ap.add_argument("--workload", default="step", choices=["step", "g_a2b"],
                    help="step: the full training step (BASELINE config 3/4); g_a2b: Generator_A2B forward + "
                         "backward only (BASELINE config 2, conv + CBAM kernels)")
    args = ap.parse_args()

    from modules import parallel
    from modules.hip import ops
    from modules.trainer import CycleGANSystem

    ops.set_mma(args.mma)
    rank, world, local = parallel.init_from_env()
    device = torch.device(f"cuda:{local}")
    torch.cuda.set_device(device)
    torch.manual_seed(1234)
    groups = args.dual and args.dual_schedule == "groups"
    if groups:
        if world < 2 or world % 2:
            raise SystemExit("--dual-schedule groups needs an even number of processes (one model per half)")
        gi, _ = parallel.split_groups(2)
        cin = (3, 2)[gi]  # soft tissue on ranks 0..w/2-1, lung on w/2..w-1
        system = CycleGANSystem(cin, args.blocks, True, device=device)
        batches = [_synthetic(args.batch, args.img, cin - 1, device, 100 * rank + i) for i in range(2)]
        step = lambda b: system.train_step(*b)
    elif args.workload == "g_a2b":
        from modules.model import Generator, weights_init_normal
        G = Generator(input_channels=args.cin, num_residual_blocks=args.blocks, use_cbam=True)
        G.apply(weights_init_normal)
        G.to(device)
        for p_ in G.parameters():
            p_.grad = torch.zeros_like(p_)
        batches = []
        for i in range(2):
            a, _, m = _synthetic(args.batch, args.img, args.cin - 1, device, 100 * rank + i)
            dout = torch.randn(args.batch, 1, args.img, args.img, device=device)
            batches.append((a, m, dout))

        def step(b):
            out = G(b[0], b[1])
            out.backward(b[2])
            return [out]
    elif args.dual:
        from modules.trainer import ConcurrentCycleGANs
        cins = (3, 2)
        runner = ConcurrentCycleGANs([CycleGANSystem(c, args.blocks, True, device=device) for c in cins], device)
        batches = [[_synthetic(args.batch, args.img, c - 1, device, 100 * rank + 10 * c + i) for c in cins]
                   for i in range(2)]
        step = lambda b: runner.train_step(b)
    else:
        system = CycleGANSystem(args.cin, args.blocks, True, device=device)
        batches = [_synthetic(args.batch, args.img, args.cin - 1, device, 100 * rank + i) for i in range(2)]
        step = lambda b: system.train_step(*b)
    models = 2 if args.dual and not groups else 1
    if args.inject_nan:
        for b in batches:
            for t in (b if args.dual and not groups else [b]):
                t[0].view(-1)[0] = float("nan")

    for i in range(args.warmup):
        step(batches[i % 2])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    ops.PROBE.reset()
    ops.PROBE.active = True
    # per-step GPU time from events at the step boundaries (no extra synchronisation): the
    # median step next to the whole-loop rate
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    marks[0].record()
    last = None
    for i in range(args.steps):
        last = step(batches[i % 2])
        marks[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    ops.PROBE.active = False
    step_ms = [marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps)]
    med_ms = statistics.median(step_ms)
    if world > 1:
        # slowest rank of the whole job (both groups of --dual-schedule groups: the default group)
        t = torch.tensor([elapsed, med_ms], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed, med_ms = float(t[0]), float(t[1])
    n_launch, ms_launch, flop_launch = ops.PROBE.summary()
    # outside the timing: the last timed step's loss terms (or Generator output) and every parameter
    # must be finite, on every rank
    outs = last if isinstance(last, (list, tuple)) else [last]
    checked = [v for o in outs for v in (o.values() if isinstance(o, dict) else [o])]
    if args.workload == "g_a2b":
        checked += [p_ for p_ in G.parameters()] + [p_.grad for p_ in G.parameters()]
    else:
        sysms_all = runner.systems if (args.dual and not groups) else [system]
        checked += [opt.flat_p for sm in sysms_all for opt in sm.optimizers]
    finite = all_finite(checked)
    if world > 1:
        fl = torch.tensor([1 if finite else 0], device=device)
        torch.distributed.all_reduce(fl, op=torch.distributed.ReduceOp.MIN)
        finite = bool(fl.item())
    replicas_ok = None
    if world > 1:  # every replica of a model must still hold the same parameters
        from modules import parallel as par
        sysms = runner.systems if (args.dual and not groups) else ([system] if args.workload == "step" else [])
        flats = [opt.flat_p for sm in sysms for opt in sm.optimizers]
        replicas_ok = par.replicas_identical(flats) if flats else None
        ok = torch.tensor([1 if replicas_ok in (True, None) else 0], device=device)
        torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN)
        replicas_ok = bool(ok.item()) if flats else None

    if rank == 0:
        # img/s over the median step; the mean over the whole timed loop beside it
        value = world * models * args.batch / (med_ms * 1e-3)
        achieved = flop_launch / (ms_launch * 1e-3) / 1e12 if ms_launch > 0 else 0.0
        pmc = _pmc_record(args.mma)
        if args.workload == "g_a2b":
            workload = ("Generator_A2B (ResNet-9 + CBAM) forward + backward (weight and input gradients), "
                        "BASELINE config 2")
        elif groups:
            workload = ("dual soft-tissue (cin 3) + lung (cin 2) CycleGANs as split GPU groups (ranks 0..w/2-1 "
                        "soft tissue, w/2..w-1 lung, one all-reduce group each), full train step per rank")
        elif args.dual:
            workload = (f"dual soft-tissue (cin 3) + lung (cin 2) CycleGANs in one process "
                        "(one after the other on one stream), "
                        "full train step per model; value = images of both models per second")
        else:
            workload = ("full soft-tissue CycleGAN train step: 2x Generator (ResNet-9 + CBAM) + 2x PatchGAN, "
                        "9 G loss terms + 2 D losses, 3 Adam steps")
        rec = {
            "metric": ("Generator_A2B fwd+bwd images/sec at 512x512 bs=8/GPU" if args.workload == "g_a2b"
                       else "CycleGAN train-step images/sec at 512x512 bs=8/GPU"),
            "value": round(value, 4),
            "unit": "img/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            # value = images / median step; ms_per_step is that median (HIP events at the step
            # boundaries), ms_per_step_mean the wall clock of the whole timed loop / steps
            "ms_per_step": round(med_ms, 3),
            "ms_per_step_median": round(med_ms, 3),
            "ms_per_step_mean": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "replicas_identical": replicas_ok,
            "finite": finite,
            "dtype": MODE_DTYPE[args.mma],
            "data": "synthetic (U(-1,1) slices, Bernoulli(0.3) masks, resident in HBM; N(0,0.02) init)",
            "config": {
                "workload": workload,
                "img_size": args.img, "per_gpu_batch": args.batch, "global_batch": args.batch * world,
                "residual_blocks": args.blocks, "input_channels": [3, 2] if args.dual else args.cin,
                "parallelism": f"2 groups x dp{world // 2}" if groups else f"dp{world}",
            },
            "roofline": {
                "kernel": ("256-ch 3x3 residual conv on the window kernel "
                           f"conv3_win16_kernel<{3 if args.mma == 'f16x3' else 1}> (v_mfma_f32_16x16x32_f16): "
                           "forward, and the data gradient's interior (+ its padded-grid ring on "
                           f"ring16_kernel<{3 if args.mma == 'f16x3' else 1}, 8> and the ring fold, inside the timed launch)"
                           if args.mma in ("f16x3", "f16") else
                           f"256-ch 3x3 residual conv rows pass: forward conv_rows_kernel<256,128,1,1,{MODE_TAG[args.mma]}>, "
                           f"data gradient conv_rows_kernel<128,128,1,1,{MODE_TAG[args.mma]}>"
                           if args.mma == "bf16x6" else
                           f"conv_rows_kernel<128,128,1,1,{MODE_TAG[args.mma]}> (256-ch 3x3 residual conv, fwd+dgrad)"),
                "bound": "mfma",
                "achieved": round(achieved, 3),
                "peak": round(MODE_PEAK[args.mma], 1),
                "unit": "TFLOP/s",
                "frac": round(achieved / MODE_PEAK[args.mma], 4),
                "traffic": pmc[0],
                "mfma_busy": pmc[1],
                "traffic_source": pmc[2],
                "launches": n_launch,
                "ms_per_launch": round(ms_launch, 4),
                "gflop_per_launch": round(flop_launch / 1e9, 3),
            },
        }
        if world == 1 and finite and not args.no_cpu_baseline and not args.dual and args.workload == "step":
            threads = min(16, os.cpu_count() or 1)
            rec["cpu_baseline"] = cpu_baseline(args.img, args.blocks, args.cin, threads)
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    if not finite:
        print("bench.py: the timed step produced non-finite losses or parameters; the record is invalid",
              file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
