# ring16 (tap split, asm B loads) tests + trace vs the rows-pass ring; wgrad staging variants by kbench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
L=$R/ducosy-gan_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_subpix.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06v_tests.log 2>&1 || { echo TESTFAIL; grep -E "^E  |FAILED" gpurun_out/r06v_tests.log | head; exit 1; }
tail -1 gpurun_out/r06v_tests.log
for it in 1 2; do
  for v in base w1 w2; do
    lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 20 --only res > gpurun_out/r06v_kb_${v}_$it.log 2>&1 || { echo "KB $v FAILED"; tail -5 gpurun_out/r06v_kb_${v}_$it.log; exit 1; }
    echo "$v/$it: $(grep -E '^res' gpurun_out/r06v_kb_${v}_$it.log | awk '{printf "%s %s  ", $2, $3}')"
  done
done
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r06v_bench.log 2>&1 || exit 1
echo "bench: $(tail -1 gpurun_out/r06v_bench.log | cut -c80-125)"
cd /tmp && export TMPDIR=/tmp
for v in base r0; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r06v_tr_$v -o tr -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/r06v_tr_$v.log 2>&1 || { echo "TRACE $v FAILED"; exit 1; }
done
echo traces ok
