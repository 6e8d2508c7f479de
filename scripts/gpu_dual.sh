set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_concurrent.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/dual_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/dual_tests.log; exit 1; }
tail -2 gpurun_out/dual_tests.log
for m in f32 bf16; do
  timeout -k 10 400 python bench.py --dual --mma $m > gpurun_out/dual_$m.log 2>&1 || { echo "dual bench $m failed"; tail -20 gpurun_out/dual_$m.log; exit 1; }
  grep -h '^{' gpurun_out/dual_$m.log | cut -c1-400
done
