set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mma.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/mma_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/mma_tests.log; exit 1; }
tail -2 gpurun_out/mma_tests.log
for m in f32 bf16 bf16x3 bf16x6; do
  timeout -k 10 200 python scripts/kbench.py --mma $m --only res,down1,down2,up1,up2,d1,d2,d3 > gpurun_out/kbench_$m.log 2>&1 || { echo "kbench $m failed"; tail -20 gpurun_out/kbench_$m.log; exit 1; }
done
paste gpurun_out/kbench_f32.log gpurun_out/kbench_bf16x3.log gpurun_out/kbench_bf16x6.log | grep -v amdgpu
