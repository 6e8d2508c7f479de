# verification at a committed HEAD: full GPU suite, smoke, default bench (cpu_baseline included), f16 and
# config-2 (g_a2b) benches, the kernel table's rocprofv3 passes (trace, FETCH_SIZE, WRITE_SIZE, MFMA busy)
# and an f16 kernel trace:  bash scripts/r05/verify.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r05v}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_full_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_full_tests.log | head -20; tail -1 gpurun_out/${T}_full_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_bench.log | cut -c1-300
timeout -k 10 300 python -u bench.py --mma f16 --no-cpu-baseline > gpurun_out/${T}_bench_f16.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_bench_f16.log | cut -c1-200
timeout -k 10 300 python -u bench.py --workload g_a2b --no-cpu-baseline > gpurun_out/${T}_bench_g_a2b.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_bench_g_a2b.log | cut -c1-200
timeout -k 10 300 python -u bench.py --dual --no-cpu-baseline --mma f16 > gpurun_out/${T}_bench_dual_f16.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_bench_dual_f16.log | cut -c1-200
bash scripts/gpu_prof_r02.sh $T || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_f16prof -o run -- python3 $R/bench.py --mma f16 --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_f16prof.log 2>&1 || exit 1
echo done
