# round-3 iteration: window tests on variant V1, kbench of every layer (default vs the variants), bench A/B
#   bash scripts/gpu_r03_step.sh V1 [V2 ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V1=$1
DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$V1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_mma.py -x -q -k "win or f16" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/st_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/st_tests.log | head -30; tail -3 gpurun_out/st_tests.log; exit 1; }
tail -1 gpurun_out/st_tests.log
bash scripts/gpu_kab.sh "" f16x3 16 "$@" || exit 1
for it in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/st_bench_A_$it.log 2>&1 || { echo BENCH A FAILED; tail -3 gpurun_out/st_bench_A_$it.log; exit 1; }
  echo "A: $(tail -1 gpurun_out/st_bench_A_$it.log | cut -c100-200)"
  for V in "$@"; do
    DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$V.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/st_bench_${V}_$it.log 2>&1 || { echo BENCH $V FAILED; tail -3 gpurun_out/st_bench_${V}_$it.log; exit 1; }
    echo "$V: $(tail -1 gpurun_out/st_bench_${V}_$it.log | cut -c100-200)"
  done
done
