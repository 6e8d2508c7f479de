# window wgrad on 16x16x32 (variant ww16) and the in-place gradient sink: tests, kbench res A/B,
# bench: A = default lib, sink off; B = default lib, sink on; C = ww16 lib, sink on; trace of C
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V=$R/ducosy-gan_amd/lib/libducosy_hip_ww16.so
DUCOSY_HIP_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_train.py tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ws_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/ws_tests.log | head -30; tail -3 gpurun_out/ws_tests.log; exit 1; }
tail -1 gpurun_out/ws_tests.log
bash scripts/gpu_kab.sh res f16x3 16 ww16 || exit 1
for it in 1 2; do
  DUCOSY_GRAD_SINK=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ws_bench_A_$it.log 2>&1 || { echo BENCH A FAILED; exit 1; }
  echo "A: $(tail -1 gpurun_out/ws_bench_A_$it.log | cut -c100-200)"
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ws_bench_B_$it.log 2>&1 || { echo BENCH B FAILED; exit 1; }
  echo "B: $(tail -1 gpurun_out/ws_bench_B_$it.log | cut -c100-200)"
  DUCOSY_HIP_LIB=$V timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ws_bench_C_$it.log 2>&1 || { echo BENCH C FAILED; exit 1; }
  echo "C: $(tail -1 gpurun_out/ws_bench_C_$it.log | cut -c100-200)"
done
cd /tmp && export TMPDIR=/tmp
DUCOSY_HIP_LIB=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ws_prof -o p --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/ws_prof.log 2>&1 || exit 1
echo prof ok
