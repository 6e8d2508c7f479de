set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tm_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/tm_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/tm_tests.log | tail -12
