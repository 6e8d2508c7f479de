set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_ops.py tests/test_gpu_mma.py tests/test_gpu_models.py tests/test_gpu_train.py > gpurun_out/d_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/d_tests.log | head -20; exit 1; }
tail -1 gpurun_out/d_tests.log
timeout -k 10 300 python scripts/kbench.py --only stem,d0 --mma bf16x6 --batch 16 --reps 7 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/d_bench.log 2>&1 || { echo BENCH FAILED; tail -5 gpurun_out/d_bench.log; exit 1; }
tail -1 gpurun_out/d_bench.log | cut -c1-250
