set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for nz in matmul wgrad; do timeout -k 10 300 python scripts/coherence_probe.py 10 $nz || exit 1; done
