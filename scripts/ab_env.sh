# A/B per-layer kernel timings with and without an environment switch, interleaved ABAB.
#   bash scripts/ab_env.sh VAR=VALUE "kbench args"
R=${GRAFT_REPO_ROOT:-$(pwd)}
SW=$1; shift
mkdir -p $R/gpurun_out
for it in 1 2; do
  echo "== A (default) round $it"
  timeout -k 10 200 python $R/scripts/kbench.py $* 2>&1 | grep -v -e amdgpu.ids -e '^layer' || exit 1
  echo "== B ($SW) round $it"
  env $SW timeout -k 10 200 python $R/scripts/kbench.py $* 2>&1 | grep -v -e amdgpu.ids -e '^layer' || exit 1
done
