# 4-channel-source x6 weight gradient (variant v4): mma / train / fullsize / models tests on it, bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V=${1:-v4}
DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$V.so timeout -k 10 500 python -u -m pytest tests/test_gpu_mma.py tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/v_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/v_tests.log | head -30; tail -3 gpurun_out/v_tests.log; exit 1; }
tail -1 gpurun_out/v_tests.log
for it in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/v_bench_A_$it.log 2>&1 || { echo BENCH A FAILED; exit 1; }
  echo "A: $(tail -1 gpurun_out/v_bench_A_$it.log | cut -c100-200)"
  DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$V.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/v_bench_B_$it.log 2>&1 || { echo BENCH B FAILED; exit 1; }
  echo "B: $(tail -1 gpurun_out/v_bench_B_$it.log | cut -c100-200)"
done
