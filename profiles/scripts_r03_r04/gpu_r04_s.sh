# f16 mode with the head / stem kernels on f16x3 operands: the two config-5 fixture tests, the head / stem tests, f16 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04s}
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_concurrent.py tests/test_gpu_train.py tests/test_gpu_head.py tests/test_gpu_stem.py > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_tests.log | head -20; tail -1 gpurun_out/${T}_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --mma f16 --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_f16.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_bench_f16.log | cut -c1-200
timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 5 --only head > gpurun_out/${T}_kbench_head.log 2>&1 || exit 1
cat gpurun_out/${T}_kbench_head.log
echo done
