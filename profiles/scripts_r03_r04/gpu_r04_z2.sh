# which parameters differ between the explicit and the autograd step with the sub-pixel window kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
echo "all";   timeout -k 10 200 python -u scripts/diag_explicit.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "fwd only"; DUCOSY_SUBWIN_DGRAD=0 timeout -k 10 200 python -u scripts/diag_explicit.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "prepack off"; DUCOSY_PREPACK=0 timeout -k 10 200 python -u scripts/diag_explicit.py 2>&1 | grep -v amdgpu.ids || exit 1
echo done
