# f16-mode tests on the default library, then f16 bench-step kernel traces, default vs variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1; shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_mma.py tests/test_gpu_concurrent.py tests/test_gpu_train.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_tests.log | head -10; tail -1 gpurun_out/${T}_tests.log
[ $rc -le 1 ] || exit 1
L=$R/ducosy-gan_amd/lib
cd /tmp && export TMPDIR=/tmp
for it in ${ITS:-1 2}; do
for v in base "$@"; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${T}_tr_${v}_$it -o tr -- python3 $R/bench.py --mma f16 --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_tr_${v}_$it.log 2>&1 || { echo "TRACE $v FAILED"; tail -3 $R/gpurun_out/${T}_tr_${v}_$it.log; exit 1; }
done
done
echo traces ok
