# sub-pixel window kernel: parity tests, up-layer kbench (window vs rows), same-box A/B (DUCOSY_SUBWIN=0|1), trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04w}
timeout -k 10 500 python -u -m pytest tests/test_gpu_subpix.py tests/test_gpu_prepack.py tests/test_gpu_train.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_tests.log | head -20; tail -1 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 24 --reps 5 --only up1,up2 > gpurun_out/${T}_kbench_up.log 2>&1 || exit 1
cat gpurun_out/${T}_kbench_up.log
for i in 1 2; do
for sw in 0 1; do
DUCOSY_SUBWIN=$sw timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_s${sw}_$i.log 2>&1 || exit 1
echo "subwin=$sw $(tail -1 gpurun_out/${T}_bench_s${sw}_$i.log | cut -c1-170)"
done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_prof.log 2>&1 || exit 1
echo done
