# f16 mode: wgrad3_win16_kernel<1> (default) vs wgrad3_win_h3_kernel<1> (w0); paired phase-kernel iterations
# (default) vs one per barrier (p0); stem / head kernels on fp16 operands (DUCOSY_F16X3_LAYERS)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
L=$R/ducosy-gan_amd/lib
timeout -k 10 900 python -u -m pytest tests/test_gpu_subpix.py tests/test_gpu_win.py tests/test_gpu_concurrent.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06ai_tests.log 2>&1 || { echo TESTFAIL; grep -E "^E  |FAILED" gpurun_out/r06ai_tests.log | head; exit 1; }
tail -1 gpurun_out/r06ai_tests.log
for v in def p0; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = def ] && lib=$L/libducosy_hip.so
  for m in f16 f16x3; do
    DUCOSY_HIP_LIB=$lib timeout -k 10 300 python -u scripts/diag/step_losses.py gpurun_out/r06ai_sl_${v}_$m.json --mma $m > gpurun_out/r06ai_sl_${v}_$m.log 2>&1 || { echo "SL $v $m FAILED"; tail -3 gpurun_out/r06ai_sl_${v}_$m.log; exit 1; }
  done
done
for m in f16 f16x3; do echo "pair vs p0 $m: $(python scripts/diag/step_losses.py --cmp gpurun_out/r06ai_sl_def_$m.json gpurun_out/r06ai_sl_p0_$m.json | tail -1)"; done
for it in 1 2; do
  for v in w0 p0 def; do
    lib=$L/libducosy_hip_$v.so; [ "$v" = def ] && lib=$L/libducosy_hip.so
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python -u scripts/kbench.py --mma f16 --batch 8 --reps 10 > gpurun_out/r06ai_kb_${v}_$it.log 2>&1 || { echo "KB $v FAILED"; exit 1; }
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --mma f16 > gpurun_out/r06ai_f16_${v}_$it.log 2>&1 || exit 1
    echo "f16 $v/$it: $(tail -1 gpurun_out/r06ai_f16_${v}_$it.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["finite"])')"
  done
done
timeout -k 10 300 python -u scripts/diag/f16_layers.py --fixed > gpurun_out/r06ai_fixed.log 2>&1 || { echo DIAG FAILED; tail -5 gpurun_out/r06ai_fixed.log; exit 1; }
grep f16x3 gpurun_out/r06ai_fixed.log
for it in 1 2; do
  for v in fx nofx; do
    fx="stem,stem_wgrad,head"; [ "$v" = nofx ] && fx=""
    DUCOSY_F16X3_LAYERS=$fx timeout -k 10 200 python bench.py --no-cpu-baseline --mma f16 > gpurun_out/r06ai_f16${v}_$it.log 2>&1 || exit 1
    echo "f16 $v/$it: $(tail -1 gpurun_out/r06ai_f16${v}_$it.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["finite"])')"
  done
done
