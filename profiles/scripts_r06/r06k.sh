set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/diag/bign_stages.py 48 > gpurun_out/r06k_stages.log 2>&1
bash scripts/pmc_stall.sh r06k16 --only res --mma f16x3 --batch 16
