# fused loss kernel + explicit step: new tests, the train/ops suites, A/B bench (explicit vs autograd step), ATen census
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_loss_fused.py tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/f_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error|^E  " gpurun_out/f_tests.log | head -30; tail -3 gpurun_out/f_tests.log; exit 1; }
tail -1 gpurun_out/f_tests.log
for it in 1 2; do
  DUCOSY_EXPLICIT_STEP=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/f_bench_A_$it.log 2>&1 || { echo BENCH A FAILED; tail -5 gpurun_out/f_bench_A_$it.log; exit 1; }
  echo "A: $(tail -1 gpurun_out/f_bench_A_$it.log | cut -c100-200)"
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/f_bench_B_$it.log 2>&1 || { echo BENCH B FAILED; tail -5 gpurun_out/f_bench_B_$it.log; exit 1; }
  echo "B: $(tail -1 gpurun_out/f_bench_B_$it.log | cut -c100-200)"
done
timeout -k 10 300 python scripts/aten_census.py > gpurun_out/aten_census2.log 2>&1 || { echo CENSUS FAILED; tail -5 gpurun_out/aten_census2.log; exit 1; }
grep -A20 "by kernel" gpurun_out/aten_census2.log | head -24
