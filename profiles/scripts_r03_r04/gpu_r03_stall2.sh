# stall breakdown of the non-residual f16x3 layers (kbench: down1, down2, up2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/pmc_stall.sh r03f --only down1,down2,up2 --mma f16x3 --batch 16 || exit 1
