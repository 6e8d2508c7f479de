# stall breakdown of the residual window kernels (kbench res, f16x3, bs 16) and the TAG-2 rows kernels (down1, up2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/pmc_stall.sh r03m --only res,down1,up2 --mma f16x3 --batch 16 || exit 1
