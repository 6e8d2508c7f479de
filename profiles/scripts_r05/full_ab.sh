# full GPU suite on the default library, then kbench (every layer) and the bench step, default vs
# each variant library, interleaved:  bash scripts/r05/full_ab.sh TAG VARIANT...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1; shift
L=$R/ducosy-gan_amd/lib
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_tests.log | head -10; tail -1 gpurun_out/${T}_tests.log
[ $rc -le 1 ] || exit 1
fi
for it in 1 2; do
  for v in base "$@"; do
    lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
    DUCOSY_HIP_LIB=$lib timeout -k 10 300 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 7 ${KB_ONLY:+--only $KB_ONLY} > gpurun_out/${T}_kb_${v}_$it.log 2>&1 || { echo "KB $v FAILED"; tail -5 gpurun_out/${T}_kb_${v}_$it.log; exit 1; }
    [ -n "$NO_BENCH" ] && continue
    DUCOSY_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_bench_${v}_$it.log 2>&1 || { echo "BENCH $v FAILED"; tail -3 gpurun_out/${T}_bench_${v}_$it.log; exit 1; }
    echo "bench $v/$it: $(tail -1 gpurun_out/${T}_bench_${v}_$it.log | cut -c60-120)"
  done
done
python scripts/r05/kb_table.py gpurun_out/${T}_kb_ base "$@"
