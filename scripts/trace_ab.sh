# Kernel traces of the bench step (rocprofv3, db output), default vs variant libraries
# (ducosy-gan_amd/lib/libducosy_hip_VARIANT.so, `make VARIANT=x EXTRA=-D...`), interleaved, plus the
# window / phase-kernel tests and one bench line per library:
#   bash scripts/trace_ab.sh TAG VARIANT...      then: python scripts/trace_cmp.py 7 gpurun_out/TAG_tr_*
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1; shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_subpix.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_tests.log | head -10; tail -1 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit 1
L=$R/ducosy-gan_amd/lib
for v in base "$@"; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench_$v.log 2>&1 || { echo "BENCH $v FAILED"; tail -3 gpurun_out/${T}_bench_$v.log; exit 1; }
  echo "bench $v: $(tail -1 gpurun_out/${T}_bench_$v.log | cut -c80-125)"
done
cd /tmp && export TMPDIR=/tmp
for it in 1 2; do
for v in base "$@"; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${T}_tr_${v}_$it -o tr -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_tr_${v}_$it.log 2>&1 || { echo "TRACE $v FAILED"; tail -3 $R/gpurun_out/${T}_tr_${v}_$it.log; exit 1; }
  echo "$v/$it: $(tail -1 $R/gpurun_out/${T}_tr_${v}_$it.log | cut -c80-125)"
done
done
echo traces ok
