# window weight gradient bring-up: its tests on the variant library, kbench A/B of the residual layer, bench A/B
#   bash scripts/gpu_r03_ww.sh VARIANT
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V=${1:-ww}
B=$R/ducosy-gan_amd/lib/libducosy_hip_$V.so
DUCOSY_HIP_LIB=$B timeout -k 10 300 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_mma.py -x -q -k "win or f16" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ww_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/ww_tests.log | head -30; tail -3 gpurun_out/ww_tests.log; exit 1; }
tail -1 gpurun_out/ww_tests.log
timeout -k 10 200 python scripts/kbench.py --batch 16 --reps 5 --mma f16x3 --only res > gpurun_out/ww_kbench_A.log 2>&1 || { echo KBENCH A FAILED; tail -5 gpurun_out/ww_kbench_A.log; exit 1; }
DUCOSY_HIP_LIB=$B timeout -k 10 200 python scripts/kbench.py --batch 16 --reps 5 --mma f16x3 --only res > gpurun_out/ww_kbench_B.log 2>&1 || { echo KBENCH B FAILED; tail -5 gpurun_out/ww_kbench_B.log; exit 1; }
echo A; cat gpurun_out/ww_kbench_A.log; echo B; cat gpurun_out/ww_kbench_B.log
for it in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ww_bench_A_$it.log 2>&1 || { echo BENCH A FAILED; tail -3 gpurun_out/ww_bench_A_$it.log; exit 1; }
  echo "A: $(tail -1 gpurun_out/ww_bench_A_$it.log | cut -c1-200)"
  DUCOSY_HIP_LIB=$B timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ww_bench_B_$it.log 2>&1 || { echo BENCH B FAILED; tail -3 gpurun_out/ww_bench_B_$it.log; exit 1; }
  echo "B: $(tail -1 gpurun_out/ww_bench_B_$it.log | cut -c1-200)"
done
