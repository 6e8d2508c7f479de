# head kernels + pre-split B: parity tests, then bench A/B (baseline / head / head + pre-split B), kernel trace, kbench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04o}
timeout -k 10 400 python -u -m pytest -v -s --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_head.py tests/test_gpu_bpre.py tests/test_gpu_stem.py > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "proj|fused|FAIL|Error" gpurun_out/${T}_tests.log | tail -30
[ $rc -le 1 ] || exit 1   # 1 = test failures (benches still informative); worse = stop
grep -E "passed|failed" gpurun_out/${T}_tests.log
for cfg in "0 0 0" "1 0 0" "1 1 0" "1 1 1"; do
  set -- $cfg
  DUCOSY_HEAD_PROJ=$1 DUCOSY_BPRE=$2 DUCOSY_STEM=$3 timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 > gpurun_out/${T}_h$1_b$2_s$3.log 2>&1 || exit 1
  echo "head=$1 bpre=$2 stem=$3 $(tail -1 gpurun_out/${T}_h$1_b$2_s$3.log | cut -c1-160)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/${T}_prof.log 2>&1 || exit 1
timeout -k 10 300 python -u $R/scripts/kbench.py --mma f16x3 --batch 16 --reps 5 > $R/gpurun_out/${T}_kbench.log 2>&1 || exit 1
cat $R/gpurun_out/${T}_kbench.log
echo done
