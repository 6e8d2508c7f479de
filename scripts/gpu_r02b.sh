set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_guard.py tests/test_gpu_concurrent.py tests/test_gpu_curve.py tests/test_gpu_fullsize.py tests/test_gpu_train.py > gpurun_out/b_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/b_tests.log; exit 1; }
grep -E "PASS|FAIL|worst" gpurun_out/b_tests.log | tail -30
timeout -k 10 300 python scripts/conc_stress.py bf16x6 30 > gpurun_out/b_stress.log 2>&1 || { echo STRESS FAILED; tail -5 gpurun_out/b_stress.log; exit 1; }
tail -1 gpurun_out/b_stress.log | cut -c1-400
timeout -k 10 300 python bench.py --workload g_a2b --steps 5 --warmup 2 > gpurun_out/b_ga2b.log 2>&1 || { echo GA2B FAILED; tail -5 gpurun_out/b_ga2b.log; exit 1; }
tail -1 gpurun_out/b_ga2b.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_bench.log 2>&1 || { echo BENCH FAILED; tail -5 gpurun_out/b_bench.log; exit 1; }
tail -1 gpurun_out/b_bench.log | cut -c1-300
