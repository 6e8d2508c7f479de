set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_x6p.py > gpurun_out/x6p_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/x6p_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/x6p_tests.log | tail
DUCOSY_X6P=0 timeout -k 10 200 python scripts/kbench.py --only res --mma bf16x6 --reps 7 > gpurun_out/x6p_kb_old.log 2>&1 || exit 1
DUCOSY_X6P=1 timeout -k 10 200 python scripts/kbench.py --only res --mma bf16x6 --reps 7 > gpurun_out/x6p_kb_new.log 2>&1 || exit 1
cat gpurun_out/x6p_kb_old.log gpurun_out/x6p_kb_new.log
cd /tmp && export TMPDIR=/tmp
DUCOSY_X6P=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/x6p_prof -o k --output-format csv -- python3 $R/scripts/kbench.py --only res --mma bf16x6 --reps 3 > $R/gpurun_out/x6p_prof.log 2>&1 || exit 1
echo prof ok
