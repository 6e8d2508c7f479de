# single-level accumulation in the residual window kernel: accuracy tests and kbench A/B (VARIANT lib)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V=$R/ducosy-gan_amd/lib/libducosy_hip_1lvl.so
DUCOSY_HIP_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_mma.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04ac_tests_1lvl.log 2>&1
echo "1lvl tests rc=$?"; grep -E "FAILED|^E  " gpurun_out/r04ac_tests_1lvl.log | head -10; tail -1 gpurun_out/r04ac_tests_1lvl.log
for i in 1 2; do
timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 5 --only res > gpurun_out/r04ac_kb_base_$i.log 2>&1 || exit 1
DUCOSY_HIP_LIB=$V timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 5 --only res > gpurun_out/r04ac_kb_1lvl_$i.log 2>&1 || exit 1
echo "base"; grep "^res" gpurun_out/r04ac_kb_base_$i.log; echo "1lvl"; grep "^res" gpurun_out/r04ac_kb_1lvl_$i.log
done
echo done
