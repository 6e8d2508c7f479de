# stride-2 window weight gradient: parity tests, kbench (window lib vs _nowin lib: x6 wgrads), same-box A/B, trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04af}
V=$R/ducosy-gan_amd/lib/libducosy_hip_nowin.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_subpix.py tests/test_gpu_train.py tests/test_gpu_models.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_tests.log | head -20; tail -1 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 5 --only down1,down2,d1,d2,d3 > gpurun_out/${T}_kbench.log 2>&1 || exit 1
DUCOSY_HIP_LIB=$V timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 5 --only down1,down2,d1,d2,d3 > gpurun_out/${T}_kbench_nowin.log 2>&1 || exit 1
echo "window"; grep wgrad gpurun_out/${T}_kbench.log; echo "x6"; grep wgrad gpurun_out/${T}_kbench_nowin.log
for i in 1 2; do
timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_new_$i.log 2>&1 || exit 1
echo "new   $(tail -1 gpurun_out/${T}_bench_new_$i.log | cut -c1-170)"
DUCOSY_HIP_LIB=$V timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_nowin_$i.log 2>&1 || exit 1
echo "nowin $(tail -1 gpurun_out/${T}_bench_nowin_$i.log | cut -c1-170)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_prof.log 2>&1 || exit 1
echo done
