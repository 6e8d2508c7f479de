set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_grads.py 2>&1 | grep -v amdgpu.ids || exit 1
echo done
