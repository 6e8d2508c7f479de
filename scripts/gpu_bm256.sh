set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_mma.py tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_train.py > gpurun_out/bm_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error|assert" gpurun_out/bm_tests.log | head -30; tail -30 gpurun_out/bm_tests.log; exit 1; }
tail -1 gpurun_out/bm_tests.log
for v in 256 128 256 128; do
  LIB=$R/ducosy-gan_amd/lib/libducosy_hip.so; [ $v = 128 ] && LIB=$R/ducosy-gan_amd/lib/libducosy_hip_bm128.so
  DUCOSY_HIP_LIB=$LIB timeout -k 10 200 python scripts/kbench.py --only res --mma bf16x6 --reps 7 > gpurun_out/bm_kb_$v.log 2>&1 || exit 1
  echo "BM $v"; grep res gpurun_out/bm_kb_$v.log | head -2
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU -d $R/gpurun_out/pmc_bm256_1 -o p --output-format csv -- python3 $R/scripts/kbench.py --only res --mma bf16x6 --reps 2 > $R/gpurun_out/pmc_bm256.log 2>&1 || exit 1
for v in 256 128; do
LIB=$R/ducosy-gan_amd/lib/libducosy_hip.so; [ $v = 128 ] && LIB=$R/ducosy-gan_amd/lib/libducosy_hip_bm128.so
DUCOSY_HIP_LIB=$LIB timeout -k 10 200 python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/bm_bench_$v.log 2>&1 || exit 1
echo "bench BM $v"; tail -1 $R/gpurun_out/bm_bench_$v.log | cut -c1-160
done
