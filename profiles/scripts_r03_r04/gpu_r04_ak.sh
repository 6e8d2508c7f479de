# fused IN-backward partial sums in the phase data gradients: parity tests, bench, trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04ak}
timeout -k 10 600 python -u -m pytest tests/test_gpu_subpix.py tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_models.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_tests.log | head -20; tail -1 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_$i.log 2>&1 || exit 1
echo "$(tail -1 gpurun_out/${T}_bench_$i.log | cut -c1-170)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_prof.log 2>&1 || exit 1
echo done
