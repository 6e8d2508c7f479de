set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u scripts/diag/bign_split.py 16 48 > gpurun_out/r06e_bign.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests -k "not config4" > gpurun_out/r06e_gpu.log 2>&1
