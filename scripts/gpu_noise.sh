set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for nz in rows wgrad; do timeout -k 10 300 python scripts/conc_noise.py bf16x6 6 $nz 300 || exit 1; done
