set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_x6p.py > gpurun_out/x6p_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/x6p_tests.log; exit 1; }
tail -1 gpurun_out/x6p_tests.log
for v in "0 1" "1 0" "1 1" "0 1" "1 0" "1 1"; do set -- $v
  DUCOSY_X6P=$1 DCS_X6P_IL=$2 timeout -k 10 200 python scripts/kbench.py --only res --mma bf16x6 --reps 7 > gpurun_out/ab_$1$2.log 2>&1 || exit 1
  echo "X6P=$1 IL=$2"; grep res gpurun_out/ab_$1$2.log
done
DUCOSY_X6P=1 DCS_X6P_IL=1 bash scripts/pmc_res.sh r02x6p "--only res --mma bf16x6" || exit 1
