# rocprofv3 evidence for the bench step at HEAD (run from the repo root on the GPU box):
# kernel trace + stats, then separate PMC passes (FETCH_SIZE; WRITE_SIZE; MFMA busy).
# BENCH_EXTRA="--mma bf16" profiles another operand mode.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_EXTRA"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_trace -o trace --output-format csv -- $B > $R/gpurun_out/prof_${TAG}_trace.log 2>&1 || exit 1
echo "trace ok"; tail -1 $R/gpurun_out/prof_${TAG}_trace.log | cut -c1-200
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_${TAG}_fetch -o fetch --output-format csv -- $B > $R/gpurun_out/prof_${TAG}_fetch.log 2>&1 || exit 1
echo "fetch ok"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_${TAG}_write -o write --output-format csv -- $B > $R/gpurun_out/prof_${TAG}_write.log 2>&1 || exit 1
echo "write ok"
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/prof_${TAG}_mfma -o mfma --output-format csv -- $B > $R/gpurun_out/prof_${TAG}_mfma.log 2>&1 || exit 1
echo "mfma ok"
