# down-conv prologue A/B on one box (DUCOSY_PRO_DOWN=0|1): subpix/fullsize tests, benches, traces
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04am}
timeout -k 10 400 python -u -m pytest tests/test_gpu_subpix.py tests/test_gpu_fullsize.py tests/test_gpu_train.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_tests.log | head -20; tail -1 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
for p in 0 1; do
DUCOSY_PRO_DOWN=$p timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_p${p}_$i.log 2>&1 || exit 1
echo "p=$p $(tail -1 gpurun_out/${T}_bench_p${p}_$i.log | cut -c1-150)"
done
done
cd /tmp && export TMPDIR=/tmp
for p in 0 1; do
DUCOSY_PRO_DOWN=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof_p$p -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_prof_p$p.log 2>&1 || exit 1
done
echo done
