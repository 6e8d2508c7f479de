# parity tests of the new head / stem / pre-split paths, then kbench (all on, then bpre off), bench, kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04p}
timeout -k 10 400 python -u -m pytest -v -s --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_head.py tests/test_gpu_bpre.py tests/test_gpu_stem.py > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "proj|fused|stem|FAIL|Error|passed|failed" gpurun_out/${T}_tests.log | tail -40
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 5 > gpurun_out/${T}_kbench.log 2>&1 || exit 1
DUCOSY_BPRE=0 timeout -k 10 300 python -u scripts/kbench.py --mma f16x3 --batch 16 --reps 5 --only down1,down2,up1,up2,d1,d2,d3 > gpurun_out/${T}_kbench_nobpre.log 2>&1 || exit 1
paste gpurun_out/${T}_kbench.log <(echo; echo; echo; echo; echo; echo; echo) | head -3 >/dev/null
cat gpurun_out/${T}_kbench.log; echo "--- bpre off"; cat gpurun_out/${T}_kbench_nobpre.log
for cfg in "0 0" "1 1"; do
  set -- $cfg
  DUCOSY_HEAD_PROJ=$1 DUCOSY_STEM=$2 timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 > gpurun_out/${T}_h$1_s$2.log 2>&1 || exit 1
  echo "head=$1 stem=$2 $(tail -1 gpurun_out/${T}_h$1_s$2.log | cut -c1-160)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/${T}_prof.log 2>&1 || exit 1
echo done
