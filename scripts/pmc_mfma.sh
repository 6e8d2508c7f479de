# MFMA-busy counters of the bench step (one PMC pass of its own, no trace domains).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01i}
MMA=${2:-f32}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_${TAG}_mfma_$MMA -o p --output-format csv \
  -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --mma $MMA > $R/gpurun_out/pmc_${TAG}_mfma_$MMA.log 2>&1 || { echo "mfma pmc failed"; tail -5 $R/gpurun_out/pmc_${TAG}_mfma_$MMA.log; exit 1; }
echo "mfma pmc $MMA ok"
