set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for m in bf16x6 f32; do echo "== $m"; timeout -k 10 300 python scripts/uninit_probe.py $m || exit 1; done
