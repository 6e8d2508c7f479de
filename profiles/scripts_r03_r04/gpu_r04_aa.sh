# full GPU suite + smoke + bench (with cpu_baseline) + kernel trace at HEAD
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04aa}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_full_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_full_tests.log | head -20; tail -1 gpurun_out/${T}_full_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_prof.log 2>&1 || exit 1
echo done
