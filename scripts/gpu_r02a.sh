# Round-2 baseline on one GPU: gpu tests, smoke, bench, PMC passes of the residual-conv kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/gpu_verify.sh || exit 1
bash scripts/pmc_res.sh r02a_x6 "--only res --mma bf16x6" || exit 1
