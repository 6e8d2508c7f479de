set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_x6p.py > gpurun_out/x6p2_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/x6p2_tests.log; exit 1; }
tail -1 gpurun_out/x6p2_tests.log
for v in 0 2 1 0 2; do
  if [ $v = 0 ]; then X=0; else X=1; fi
  DUCOSY_X6P=$X DCS_X6P_VARIANT=$v timeout -k 10 200 python scripts/kbench.py --only res --mma bf16x6 --reps 7 > gpurun_out/ab2_$v.log 2>&1 || exit 1
  echo "variant $v"; grep res gpurun_out/ab2_$v.log | head -2
done
DUCOSY_X6P=1 DCS_X6P_VARIANT=2 bash scripts/pmc_res.sh r02x6p2 "--only res --mma bf16x6" || exit 1
