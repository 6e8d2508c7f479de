# full GPU suite, smoke and the default bench at HEAD; then the f16 operand mode (config 5's path): bench + kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04r}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_full_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_full_tests.log | head -20; tail -1 gpurun_out/${T}_full_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH FAILED; tail -5 gpurun_out/${T}_bench.log; exit 1; }
tail -1 gpurun_out/${T}_bench.log | cut -c1-300
timeout -k 10 300 python bench.py --mma f16 --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_f16.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_bench_f16.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof_f16 -o run -- python3 $R/bench.py --mma f16 --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_prof_f16.log 2>&1 || exit 1
echo done
