set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/diag/bign_stages.py 48 > gpurun_out/r06g_stages.log 2>&1
bash scripts/r06h.sh
