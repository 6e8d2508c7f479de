# A/B of the 7x7 head forward: tap projection on MFMA (DUCOSY_HEAD_PROJ=1) vs the VALU kernel, then a kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04n}
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_head.py > gpurun_out/${T}_head.log 2>&1 || { tail -30 gpurun_out/${T}_head.log; exit 1; }
grep -E "proj|passed|failed" gpurun_out/${T}_head.log
for p in 0 1; do
  DUCOSY_HEAD_PROJ=$p timeout -k 10 240 python -u bench.py --steps 12 --warmup 3 > gpurun_out/${T}_proj$p.log 2>&1 || exit 1
  echo "proj=$p $(tail -1 gpurun_out/${T}_proj$p.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/${T}_prof.log 2>&1 || exit 1
timeout -k 10 300 python -u $R/scripts/kbench.py --mma f16x3 --batch 16 --reps 5 > $R/gpurun_out/${T}_kbench.log 2>&1 || exit 1
cat $R/gpurun_out/${T}_kbench.log
echo done
