# quick GPU check: op / model / train / full-size parity tests, then one bench line
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_train.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/q_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/q_tests.log | head -20; exit 1; }
tail -1 gpurun_out/q_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/q_bench.log 2>&1 || { echo BENCH FAILED; tail -3 gpurun_out/q_bench.log; exit 1; }
tail -1 gpurun_out/q_bench.log | cut -c1-150
