set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for v in 3 1; do
DUCOSY_X6P=1 DCS_X6P_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_x6p.py > gpurun_out/x6p3_tests_$v.log 2>&1 || { echo TESTS FAILED $v; tail -40 gpurun_out/x6p3_tests_$v.log; exit 1; }
tail -1 gpurun_out/x6p3_tests_$v.log
done
for v in 0 3 1 0 3; do
  if [ $v = 0 ]; then X=0; else X=1; fi
  DUCOSY_X6P=$X DCS_X6P_VARIANT=$v timeout -k 10 200 python scripts/kbench.py --only res --mma bf16x6 --reps 7 > gpurun_out/ab3_$v.log 2>&1 || exit 1
  echo "variant $v"; grep res gpurun_out/ab3_$v.log | head -2
done
cd /tmp && export TMPDIR=/tmp
DUCOSY_X6P=1 DCS_X6P_VARIANT=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/x6p3_prof -o k --output-format csv -- python3 $R/scripts/kbench.py --only res --mma bf16x6 --reps 3 > $R/gpurun_out/x6p3_prof.log 2>&1 || exit 1
cd $R && DUCOSY_X6P=1 DCS_X6P_VARIANT=3 bash scripts/pmc_res.sh r02x6p3 "--only res --mma bf16x6" || exit 1
