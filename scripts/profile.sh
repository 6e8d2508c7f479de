# rocprofv3 evidence for the bench workload (run from the repo root on the GPU box).
#   kernel trace + stats, then separate PMC passes for FETCH_SIZE and WRITE_SIZE.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
MMA=${2:-bf16x6}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_${MMA}_trace -o trace --output-format csv \
  -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --mma $MMA > $R/gpurun_out/prof_${TAG}_${MMA}_trace.log 2>&1 || exit $?
echo "trace ok"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_${TAG}_${MMA}_fetch -o fetch --output-format csv \
  -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --mma $MMA > $R/gpurun_out/prof_${TAG}_${MMA}_fetch.log 2>&1 || exit $?
echo "fetch ok"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_${TAG}_${MMA}_write -o write --output-format csv \
  -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --mma $MMA > $R/gpurun_out/prof_${TAG}_${MMA}_write.log 2>&1 || exit $?
echo "write ok"
