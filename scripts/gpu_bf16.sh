# half-precision (config 5) path: operand-mode tests, bf16 bench line, bf16 kernel profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mma.py tests/test_gpu_train.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/bf16_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/bf16_tests.log | head -20; exit 1; }
tail -1 gpurun_out/bf16_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --mma bf16 > gpurun_out/bf16_bench.log 2>&1 || { echo BENCH FAILED; tail -3 gpurun_out/bf16_bench.log; exit 1; }
echo "bf16: $(tail -1 gpurun_out/bf16_bench.log | cut -c80-130)"
timeout -k 10 300 python bench.py --no-cpu-baseline --dual --mma bf16 > gpurun_out/bf16_dual_bench.log 2>&1 || { echo BENCH FAILED; tail -3 gpurun_out/bf16_dual_bench.log; exit 1; }
echo "bf16 dual: $(tail -1 gpurun_out/bf16_dual_bench.log | cut -c80-130)"
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/x6_bench.log 2>&1 || { echo BENCH FAILED; tail -3 gpurun_out/x6_bench.log; exit 1; }
echo "bf16x6: $(tail -1 gpurun_out/x6_bench.log | cut -c80-130)"
BENCH_EXTRA="--mma bf16" bash scripts/gpu_prof_r02.sh r02g_bf16
