# fp16 mode: the stride-2 window kernels on fp16 operands (up-convs stay f16x3): fixture tests, f16 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04ah}
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_concurrent.py tests/test_gpu_subpix.py tests/test_gpu_precision.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_tests.log | head -20; tail -1 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 240 python -u bench.py --mma f16 --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_f16_$i.log 2>&1 || exit 1
echo "f16 $(tail -1 gpurun_out/${T}_bench_f16_$i.log | cut -c1-170)"
done
echo done
