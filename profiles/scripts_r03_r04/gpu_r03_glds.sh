# LDS-DMA B staging in the window kernels (variant glds): window / ops / train tests on it, kbench res A/B x2, bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V=${1:-glds}
DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/g_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/g_tests.log | head -30; tail -3 gpurun_out/g_tests.log; exit 1; }
tail -1 gpurun_out/g_tests.log
bash scripts/gpu_kab.sh res f16x3 16 $V || exit 1
bash scripts/gpu_kab.sh res f16x3 16 $V || exit 1
for it in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/g_bench_A_$it.log 2>&1 || { echo BENCH A FAILED; exit 1; }
  echo "A: $(tail -1 gpurun_out/g_bench_A_$it.log | cut -c100-200)"
  DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$V.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/g_bench_B_$it.log 2>&1 || { echo BENCH B FAILED; exit 1; }
  echo "B: $(tail -1 gpurun_out/g_bench_B_$it.log | cut -c100-200)"
done
