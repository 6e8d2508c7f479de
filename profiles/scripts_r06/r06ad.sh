# window conv unit loads as asm with explicit vmcnt (base, DCS_WIN_ASYNC=1) vs compiler-tracked (sync)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
L=$R/ducosy-gan_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_fullsize.py -q -x --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/r06ad_tests.log 2>&1 || { echo TESTFAIL; grep -E "^E  |FAILED" gpurun_out/r06ad_tests.log | head; exit 1; }
tail -1 gpurun_out/r06ad_tests.log
for it in 1 2; do
  for v in base sync; do
    lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 20 --only res > gpurun_out/r06ad_kb_${v}_$it.log 2>&1 || { echo "KB $v FAILED"; exit 1; }
    echo "$v/$it: $(grep -E '^res' gpurun_out/r06ad_kb_${v}_$it.log | awk '{printf "%s %s  ", $2, $3}')"
  done
done
for it in 1 2; do
  for v in base sync; do
    lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r06ad_bench_${v}_$it.log 2>&1 || exit 1
    echo "bench $v/$it: $(tail -1 gpurun_out/r06ad_bench_${v}_$it.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["ms_per_launch"], d["finite"])')"
  done
done
