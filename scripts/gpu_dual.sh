# Config 5 (soft-tissue + lung models in one process): runner tests, then the dual bench in
# both schedules (serial: one stream, default bf16x6; concurrent: two streams, exact f32).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_concurrent.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/dual_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/dual_tests.log; exit 1; }
tail -2 gpurun_out/dual_tests.log
for sch in serial concurrent; do
  timeout -k 10 400 python bench.py --dual --dual-schedule $sch --no-cpu-baseline > gpurun_out/dual_$sch.log 2>&1 || { echo "dual bench $sch failed"; tail -20 gpurun_out/dual_$sch.log; exit 1; }
  grep -h '^{' gpurun_out/dual_$sch.log | cut -c1-330
done
