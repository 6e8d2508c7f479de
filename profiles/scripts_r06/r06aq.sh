# f16 PatchGAN weight gradients on the LeakyReLU-prologue x6 instance (TAG 3, default) vs the generic one (t0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
L=$R/ducosy-gan_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_subpix.py tests/test_gpu_concurrent.py tests/test_gpu_mma.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06aq_tests.log 2>&1 || { echo TESTFAIL; grep -E "^E  |FAILED" gpurun_out/r06aq_tests.log | head; exit 1; }
tail -1 gpurun_out/r06aq_tests.log
for v in def t0; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = def ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 300 python -u scripts/diag/step_losses.py gpurun_out/r06aq_sl_$v.json --mma f16 > gpurun_out/r06aq_sl_$v.log 2>&1 || { echo "SL $v FAILED"; exit 1; }
done
echo "tag3 vs t0 f16: $(python scripts/diag/step_losses.py --cmp gpurun_out/r06aq_sl_def.json gpurun_out/r06aq_sl_t0.json | tail -1)"
for it in 1 2; do
  for v in t0 def; do
    lib=$L/libducosy_hip_$v.so; [ "$v" = def ] && lib=$L/libducosy_hip.so
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python -u scripts/kbench.py --mma f16 --batch 8 --reps 10 --only d1,d2,d3 > gpurun_out/r06aq_kb_${v}_$it.log 2>&1 || { echo "KB $v FAILED"; exit 1; }
    echo "$v/$it: $(grep -E 'wgrad' gpurun_out/r06aq_kb_${v}_$it.log | awk '{printf "%s/%s %s  ", $1, $2, $3}')"
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --mma f16 > gpurun_out/r06aq_f16_${v}_$it.log 2>&1 || exit 1
    echo "f16 $v/$it: $(tail -1 gpurun_out/r06aq_f16_${v}_$it.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["finite"])')"
  done
done
