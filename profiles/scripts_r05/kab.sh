# A/B of library variants on the residual conv kernels (kbench res at bs 16 = the bench's batched
# calls), interleaved; window tests per variant.
#   bash scripts/r05/kab.sh TAG VARIANT...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1; shift
L=$R/ducosy-gan_amd/lib
for v in "$@"; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_win.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_test_$v.log 2>&1 || { echo "TEST $v FAILED"; grep -E "^E  " gpurun_out/${T}_test_$v.log | head -4; }
  echo "tests $v: $(tail -1 gpurun_out/${T}_test_$v.log)"
done
for it in 1 2; do
  for v in "$@"; do
    lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 9 --only res > gpurun_out/${T}_kb_${v}_$it.log 2>&1 || { echo "KB $v FAILED"; tail -5 gpurun_out/${T}_kb_${v}_$it.log; exit 1; }
    echo "$v/$it: $(grep -E '^res' gpurun_out/${T}_kb_${v}_$it.log | awk '{printf "%s %s  ", $2, $3}')"
  done
done
