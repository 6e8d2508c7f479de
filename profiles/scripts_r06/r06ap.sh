# f16 residual weight gradient with fragment reuse (each B fragment feeds both co blocks; default) vs
# wgrad3_win_h3_kernel<1> (r0 lib)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
L=$R/ducosy-gan_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_concurrent.py tests/test_gpu_fullsize.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06ap_tests.log 2>&1 || { echo TESTFAIL; grep -E "^E  |FAILED" gpurun_out/r06ap_tests.log | head; exit 1; }
tail -1 gpurun_out/r06ap_tests.log
for it in 1 2; do
  for v in r0 def; do
    lib=$L/libducosy_hip_$v.so; [ "$v" = def ] && lib=$L/libducosy_hip.so
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python -u scripts/kbench.py --mma f16 --batch 16 --reps 20 --only res > gpurun_out/r06ap_kb_${v}_$it.log 2>&1 || { echo "KB $v FAILED"; exit 1; }
    echo "$v/$it: $(grep -E '^res' gpurun_out/r06ap_kb_${v}_$it.log | awk '{printf "%s %s  ", $2, $3}')"
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --mma f16 > gpurun_out/r06ap_f16_${v}_$it.log 2>&1 || exit 1
    echo "f16 $v/$it: $(tail -1 gpurun_out/r06ap_f16_${v}_$it.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["finite"])')"
  done
done
