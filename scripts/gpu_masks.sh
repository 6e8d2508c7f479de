set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_masks.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/m_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/m_tests.log; exit 1; }
tail -3 gpurun_out/m_tests.log
timeout -k 10 120 python scripts/bench_masks.py > gpurun_out/m_bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/m_bench.log; exit 1; }
timeout -k 10 120 python scripts/bench_masks.py --kinds lung,mediastinum,bone,lung_vessel >> gpurun_out/m_bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/m_bench.log; exit 1; }
cat gpurun_out/m_bench.log | grep -v amdgpu.ids
