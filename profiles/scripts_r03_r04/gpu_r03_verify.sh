# round-3 verification at HEAD: full GPU suite, smoke, bench (with CPU baseline), then the kernel table passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/gpu_full.sh || exit 1
bash scripts/gpu_prof_r02.sh ${1:-r03k} || exit 1
