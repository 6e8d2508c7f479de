# f16x3 bring-up: fp16 MFMA denormal probe, operand-mode precision tests, bf16x6 vs f16x3 bench
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 60 ./scripts/probes/f16_denorm > gpurun_out/f16_denorm.log 2>&1; cat gpurun_out/f16_denorm.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_mma.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mma_tests.log 2>&1 || { echo MMA TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/mma_tests.log | head -30; exit 1; }
tail -1 gpurun_out/mma_tests.log
for m in bf16x6 f16x3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --mma $m --steps 5 --warmup 2 > gpurun_out/bench_$m.log 2>&1 || { echo BENCH $m FAILED; tail -5 gpurun_out/bench_$m.log; exit 1; }
  echo "$m: $(tail -1 gpurun_out/bench_$m.log | cut -c1-200)"
done
