set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/profile.sh r01i || exit 1
bash scripts/pmc_mfma.sh r01i f32 || exit 1
bash scripts/pmc_mfma.sh r01i bf16 || exit 1
echo all ok
