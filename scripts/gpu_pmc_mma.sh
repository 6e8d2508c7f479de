set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/pmc_res.sh resf32 --only res --mma f32 || exit 1
bash scripts/pmc_res.sh resbf16 --only res --mma bf16 || exit 1
echo pmc both ok
