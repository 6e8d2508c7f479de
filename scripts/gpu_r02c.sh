# narrow data-gradient kernels: parity tests, bench, kernel trace of the bench step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTS:-tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_train.py tests/test_gpu_dataset.py tests/test_gpu_fullsize.py} > gpurun_out/c_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error|assert" gpurun_out/c_tests.log | head -20; tail -30 gpurun_out/c_tests.log; exit 1; }
tail -2 gpurun_out/c_tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c_bench.log 2>&1 || { echo BENCH FAILED; tail -5 gpurun_out/c_bench.log; exit 1; }
tail -1 gpurun_out/c_bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c_trace -o trace --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_c_trace.log 2>&1 || { echo PROF FAILED; exit 1; }
echo prof ok
