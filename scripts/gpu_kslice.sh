# slice-major K order of the residual convs: parity tests, kernel A/B, L2 counters
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_mma.py tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_x6p.py tests/test_gpu_precision.py tests/test_gpu_train.py > gpurun_out/ks_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error|assert" gpurun_out/ks_tests.log | head -30; tail -30 gpurun_out/ks_tests.log; exit 1; }
tail -1 gpurun_out/ks_tests.log
for k in 1 0 1 0; do
  DUCOSY_KSLICE=$k timeout -k 10 200 python scripts/kbench.py --only res --mma bf16x6 --reps 7 > gpurun_out/ks_kb_$k.log 2>&1 || exit 1
  echo "KSLICE=$k"; grep res gpurun_out/ks_kb_$k.log
done
DUCOSY_KSLICE=1 timeout -k 10 200 python scripts/kbench.py --only res --mma f32 --reps 5 > gpurun_out/ks_kb_f32.log 2>&1 || exit 1
echo "f32 KSLICE=1"; grep res gpurun_out/ks_kb_f32.log
cd /tmp && export TMPDIR=/tmp
for k in 1 0; do
DUCOSY_KSLICE=$k timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc_ks${k}_1 -o p --output-format csv -- python3 $R/scripts/kbench.py --only res --mma bf16x6 --reps 2 > $R/gpurun_out/pmc_ks$k.log 2>&1 || exit 1
DUCOSY_KSLICE=$k timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_ks${k}_2 -o p --output-format csv -- python3 $R/scripts/kbench.py --only res --mma bf16x6 --reps 2 > $R/gpurun_out/pmc_ks${k}b.log 2>&1 || exit 1
done
echo pmc ok
