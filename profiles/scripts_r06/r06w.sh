# ring16 with four k-steps in flight; wgrad staging variants (w1: pieces in k-step 2 at 1/3/5, w3: 3/5/7)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
L=$R/ducosy-gan_amd/lib
for v in base w1; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_subpix.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06w_tests_$v.log 2>&1 || { echo "TESTFAIL $v"; grep -E "^E  |FAILED" gpurun_out/r06w_tests_$v.log | head; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/r06w_tests_$v.log)"
done
for it in 1 2; do
  for v in base w1 w3; do
    lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 20 --only res > gpurun_out/r06w_kb_${v}_$it.log 2>&1 || { echo "KB $v FAILED"; tail -5 gpurun_out/r06w_kb_${v}_$it.log; exit 1; }
    echo "$v/$it: $(grep -E '^res' gpurun_out/r06w_kb_${v}_$it.log | awk '{printf "%s %s  ", $2, $3}')"
  done
done
for v in base w1; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r06w_bench_$v.log 2>&1 || exit 1
  echo "bench $v: $(tail -1 gpurun_out/r06w_bench_$v.log | cut -c80-125)"
done
cd /tmp && export TMPDIR=/tmp
for v in base r0; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r06w_tr_$v -o tr -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/r06w_tr_$v.log 2>&1 || { echo "TRACE $v FAILED"; exit 1; }
done
echo traces ok
