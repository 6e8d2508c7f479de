# stem pre-split window + faster reduces; NSUB = 2 for 64-column f16x3 rows tiles (variant library): parity, kbench, bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04q}
V=$R/ducosy-gan_amd/lib/libducosy_hip_nsub64.so
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_stem.py tests/test_gpu_head.py > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAIL" gpurun_out/${T}_tests.log | tail -8
[ $rc -le 1 ] || exit 1
DUCOSY_HIP_LIB=$V timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_mma.py tests/test_gpu_bpre.py tests/test_gpu_ops.py > gpurun_out/${T}_tests_nsub64.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests_nsub64.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 5 --only stem,down1,up2,d1,head > gpurun_out/${T}_kbench.log 2>&1 || exit 1
DUCOSY_HIP_LIB=$V timeout -k 10 300 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 5 --only down1,up2,d1 > gpurun_out/${T}_kbench_nsub64.log 2>&1 || exit 1
cat gpurun_out/${T}_kbench.log; echo "--- nsub64"; cat gpurun_out/${T}_kbench_nsub64.log
timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 > gpurun_out/${T}_bench.log 2>&1 || exit 1
echo "default $(tail -1 gpurun_out/${T}_bench.log | cut -c1-160)"
DUCOSY_HIP_LIB=$V timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 > gpurun_out/${T}_bench_nsub64.log 2>&1 || exit 1
echo "nsub64 $(tail -1 gpurun_out/${T}_bench_nsub64.log | cut -c1-160)"
echo done
