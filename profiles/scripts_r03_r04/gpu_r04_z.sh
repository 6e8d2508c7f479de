# sub-pixel window dgrad + wgrad: parity tests, explicit-vs-autograd margins (subwin on / off), kbench,
# same-box A/B: new lib / lib without the window wgrad (_nosw) / new lib with DUCOSY_SUBWIN=0
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04z}
timeout -k 10 300 python -u -m pytest tests/test_gpu_subpix.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_tests.log | head -20; tail -1 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit 1
echo "subwin=1"; timeout -k 10 200 python -u scripts/diag_explicit.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "subwin=0"; DUCOSY_SUBWIN=0 timeout -k 10 200 python -u scripts/diag_explicit.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "nosw lib"; DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_nosw.so timeout -k 10 200 python -u scripts/diag_explicit.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 5 --only up1,up2 > gpurun_out/${T}_kbench.log 2>&1 || exit 1
cat gpurun_out/${T}_kbench.log
DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_nosw.so timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 5 --only up1,up2 > gpurun_out/${T}_kbench_nosw.log 2>&1 || exit 1
grep wgrad gpurun_out/${T}_kbench_nosw.log
for i in 1 2; do
timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_new_$i.log 2>&1 || exit 1
echo "new     $(tail -1 gpurun_out/${T}_bench_new_$i.log | cut -c1-170)"
DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_nosw.so timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_nosw_$i.log 2>&1 || exit 1
echo "nosw    $(tail -1 gpurun_out/${T}_bench_nosw_$i.log | cut -c1-170)"
DUCOSY_SUBWIN=0 timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_s0_$i.log 2>&1 || exit 1
echo "subwin0 $(tail -1 gpurun_out/${T}_bench_s0_$i.log | cut -c1-170)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_prof.log 2>&1 || exit 1
echo done
