# stall breakdown of the f16x3 residual kernels (kbench) + the bench-step kernel table passes
#   bash scripts/gpu_r03_prof.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/pmc_stall.sh ${1}res --only res --mma f16x3 --batch 16 || exit 1
bash scripts/gpu_prof_r02.sh $1 || exit 1
