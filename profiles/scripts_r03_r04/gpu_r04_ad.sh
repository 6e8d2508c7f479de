# stride-2 window phase kernels (down-convs + PatchGAN layers): parity tests, kbench, same-box A/B (DUCOSY_S2WIN=0|1), trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04ad}
timeout -k 10 600 python -u -m pytest tests/test_gpu_subpix.py tests/test_gpu_bpre.py tests/test_gpu_prepack.py tests/test_gpu_train.py tests/test_gpu_models.py tests/test_gpu_fullsize.py tests/test_gpu_concurrent.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_tests.log | head -20; tail -1 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 5 --only d1,d2,d3,down1,down2 > gpurun_out/${T}_kbench.log 2>&1 || exit 1
cat gpurun_out/${T}_kbench.log
for i in 1 2; do
for sw in 1 0; do
DUCOSY_S2WIN=$sw timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_s${sw}_$i.log 2>&1 || exit 1
echo "s2win=$sw $(tail -1 gpurun_out/${T}_bench_s${sw}_$i.log | cut -c1-170)"
done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_prof.log 2>&1 || exit 1
echo done
