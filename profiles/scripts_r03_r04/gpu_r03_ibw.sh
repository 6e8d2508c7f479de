# fused IN-backward partial sums (window data gradient epilogue + ring fold) and the gradient sink:
# tests, bench A/B (DUCOSY_FUSE_IBW 0 / 1), kernel trace of the fused step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_models.py tests/test_gpu_train.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ib_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/ib_tests.log | head -30; tail -3 gpurun_out/ib_tests.log; exit 1; }
tail -1 gpurun_out/ib_tests.log
for it in 1 2; do
  for f in 0 1; do
    DUCOSY_FUSE_IBW=$f timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ib_bench_${f}_$it.log 2>&1 || { echo BENCH $f FAILED; exit 1; }
    echo "ibw=$f: $(tail -1 gpurun_out/ib_bench_${f}_$it.log | cut -c100-200)"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ib_prof -o p --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/ib_prof.log 2>&1 || exit 1
echo prof ok
