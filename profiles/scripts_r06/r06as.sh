# f16 stride-2 data gradient, column phase 0, with two window register sets (default) vs one (w1 lib)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
L=$R/ducosy-gan_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_subpix.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06as_tests.log 2>&1 || { echo TESTFAIL; grep -E "^E  |FAILED" gpurun_out/r06as_tests.log | head; exit 1; }
tail -1 gpurun_out/r06as_tests.log
for v in def w1; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = def ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 300 python -u scripts/diag/step_losses.py gpurun_out/r06as_sl_$v.json --mma f16 > gpurun_out/r06as_sl_$v.log 2>&1 || { echo "SL $v FAILED"; exit 1; }
done
echo "wr2 vs w1 f16: $(python scripts/diag/step_losses.py --cmp gpurun_out/r06as_sl_def.json gpurun_out/r06as_sl_w1.json | tail -1)"
for it in 1 2; do
  for v in w1 def; do
    lib=$L/libducosy_hip_$v.so; [ "$v" = def ] && lib=$L/libducosy_hip.so
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python -u scripts/kbench.py --mma f16 --batch 8 --reps 10 --only down1,down2,d1,d2,d3 > gpurun_out/r06as_kb_${v}_$it.log 2>&1 || { echo "KB $v FAILED"; exit 1; }
    echo "$v/$it: $(grep -E 'dgrad' gpurun_out/r06as_kb_${v}_$it.log | awk '{printf "%s/%s %s  ", $1, $2, $3}')"
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --mma f16 > gpurun_out/r06as_f16_${v}_$it.log 2>&1 || exit 1
    echo "f16 $v/$it: $(tail -1 gpurun_out/r06as_f16_${v}_$it.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["finite"])')"
  done
done
