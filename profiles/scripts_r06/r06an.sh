# f16 residual weight gradient: both rows of the next barrier loaded at its start, one accumulation level
# (default) vs each row's loads at its start (e0 lib)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
L=$R/ducosy-gan_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_concurrent.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06an_tests.log 2>&1 || { echo TESTFAIL; grep -E "^E  |FAILED" gpurun_out/r06an_tests.log | head; exit 1; }
tail -1 gpurun_out/r06an_tests.log
for it in 1 2; do
  for v in e0 def; do
    lib=$L/libducosy_hip_$v.so; [ "$v" = def ] && lib=$L/libducosy_hip.so
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python -u scripts/kbench.py --mma f16 --batch 16 --reps 20 --only res > gpurun_out/r06an_kb_${v}_$it.log 2>&1 || { echo "KB $v FAILED"; exit 1; }
    echo "$v/$it: $(grep -E '^res' gpurun_out/r06an_kb_${v}_$it.log | awk '{printf "%s %s  ", $2, $3}')"
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --mma f16 > gpurun_out/r06an_f16_${v}_$it.log 2>&1 || exit 1
    echo "f16 $v/$it: $(tail -1 gpurun_out/r06an_f16_${v}_$it.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["finite"])')"
  done
done
