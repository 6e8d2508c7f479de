# tests (win, mma, concurrent, train, subpix) on the default library, then bench-step kernel traces in
# f16x3 and f16, default vs variants:  bash scripts/r05/both_ab.sh TAG VARIANT...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1; shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_mma.py tests/test_gpu_concurrent.py tests/test_gpu_train.py tests/test_gpu_subpix.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_tests.log | head -10; tail -1 gpurun_out/${T}_tests.log
[ $rc -le 1 ] || exit 1
L=$R/ducosy-gan_amd/lib
cd /tmp && export TMPDIR=/tmp
for mode in f16x3 f16; do
for v in base "$@"; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${T}_${mode}_${v} -o tr -- python3 $R/bench.py --mma $mode --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_${mode}_${v}.log 2>&1 || { echo "TRACE $v FAILED"; tail -3 $R/gpurun_out/${T}_${mode}_${v}.log; exit 1; }
done
done
cd $R
for mode in f16x3 f16; do
  dirs=""; for v in base "$@"; do dirs="$dirs gpurun_out/${T}_${mode}_${v}"; done
  python scripts/r05/trace_cmp.py 7 $dirs > gpurun_out/${T}_cmp_${mode}.txt || exit 1
  for k in ${INST:-}; do python scripts/r05/trace_inst.py 7 $k $dirs > gpurun_out/${T}_inst_${k}_${mode}.txt || exit 1; done
  rm -rf $dirs  # the databases exceed what gpurun copies back; the table is the record
done
echo traces ok
