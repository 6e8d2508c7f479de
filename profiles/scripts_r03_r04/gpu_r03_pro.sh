# IN-apply prologue fusion: window / model / train / fullsize tests, bench A/B by DUCOSY_FUSE_PRO
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_models.py tests/test_gpu_train.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/p_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/p_tests.log | head -30; tail -3 gpurun_out/p_tests.log; exit 1; }
tail -1 gpurun_out/p_tests.log
for it in 1 2; do
  DUCOSY_FUSE_PRO=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/p_bench_A_$it.log 2>&1 || { echo BENCH A FAILED; exit 1; }
  echo "A: $(tail -1 gpurun_out/p_bench_A_$it.log | cut -c100-200)"
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/p_bench_B_$it.log 2>&1 || { echo BENCH B FAILED; exit 1; }
  echo "B: $(tail -1 gpurun_out/p_bench_B_$it.log | cut -c100-200)"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --mma f16 > gpurun_out/p_bench_f16.log 2>&1 || { echo BENCH f16 FAILED; exit 1; }
echo "f16: $(tail -1 gpurun_out/p_bench_f16.log | cut -c1-900)"
