# stall counters of the f16 residual kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/pmc_stall.sh r05p --only res --mma f16 --batch 16 || exit 1
