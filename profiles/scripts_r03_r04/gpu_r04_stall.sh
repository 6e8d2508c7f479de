# stall counters of the window kernels, v2 and v1 (kbench res, f16x3, bs 16)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/pmc_stall.sh ${1}v2 --only res --mma f16x3 --batch 16 || exit 1
DCS_WIN_V1=1 bash scripts/pmc_stall.sh ${1}v1 --only res --mma f16x3 --batch 16 || exit 1
