# full GPU suite + head kbench + bench: smaller pack grids, branch-free border entries in the fused head backward
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04t}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_full_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_full_tests.log | head -20; tail -1 gpurun_out/${T}_full_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 5 --only head > gpurun_out/${T}_kbench_head.log 2>&1 || exit 1
cat gpurun_out/${T}_kbench_head.log
timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_prof.log 2>&1 || exit 1
echo done
