set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/profile.sh ${TAG:-r01k} bf16x6 || exit 1
bash scripts/pmc_mfma.sh ${TAG:-r01k} bf16x6 || exit 1
echo all ok
