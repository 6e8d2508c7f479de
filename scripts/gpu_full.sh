# full GPU suite, smoke, bench (with CPU baseline) and a kernel trace of the bench step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/full_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/full_tests.log | head -20; tail -5 gpurun_out/full_tests.log; exit 1; }
tail -1 gpurun_out/full_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full_smoke.log 2>&1 || { echo SMOKE FAILED; tail -5 gpurun_out/full_smoke.log; exit 1; }
tail -1 gpurun_out/full_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/full_bench.log 2>&1 || { echo BENCH FAILED; tail -5 gpurun_out/full_bench.log; exit 1; }
tail -1 gpurun_out/full_bench.log | cut -c1-400
