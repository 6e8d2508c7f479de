# Round-end style verification on one GPU: gpu tests, smoke, default bench (with CPU baseline).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/v_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/v_tests.log; exit 1; }
tail -3 gpurun_out/v_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/v_smoke.log; exit 1; }
tail -2 gpurun_out/v_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/v_bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/v_bench.log; exit 1; }
tail -2 gpurun_out/v_bench.log
