# window phase kernels: B slices by LDS-DMA with unconditional window stores (default) vs registers + ds_write
# (nb lib): phase-kernel tests, bit-exactness of three f16 / f16x3 steps, kbench, f16x3 and f16 benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
L=$R/ducosy-gan_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_subpix.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06ak_tests.log 2>&1 || { echo TESTFAIL; grep -E "^E  |FAILED" gpurun_out/r06ak_tests.log | head; exit 1; }
tail -1 gpurun_out/r06ak_tests.log
for v in def nb; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = def ] && lib=$L/libducosy_hip.so
  for m in f16 f16x3; do
    DUCOSY_HIP_LIB=$lib timeout -k 10 300 python -u scripts/diag/step_losses.py gpurun_out/r06ak_sl_${v}_$m.json --mma $m > gpurun_out/r06ak_sl_${v}_$m.log 2>&1 || { echo "SL $v $m FAILED"; tail -3 gpurun_out/r06ak_sl_${v}_$m.log; exit 1; }
  done
done
for m in f16 f16x3; do echo "bdma vs nb $m: $(python scripts/diag/step_losses.py --cmp gpurun_out/r06ak_sl_def_$m.json gpurun_out/r06ak_sl_nb_$m.json | tail -1)"; done
for it in 1 2; do
  for v in nb def; do
    lib=$L/libducosy_hip_$v.so; [ "$v" = def ] && lib=$L/libducosy_hip.so
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python -u scripts/kbench.py --batch 8 --reps 10 > gpurun_out/r06ak_kb_${v}_$it.log 2>&1 || { echo "KB $v FAILED"; exit 1; }
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r06ak_b_${v}_$it.log 2>&1 || exit 1
    echo "f16x3 $v/$it: $(tail -1 gpurun_out/r06ak_b_${v}_$it.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["finite"])')"
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --mma f16 > gpurun_out/r06ak_f16_${v}_$it.log 2>&1 || exit 1
    echo "f16 $v/$it: $(tail -1 gpurun_out/r06ak_f16_${v}_$it.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["finite"])')"
  done
done
