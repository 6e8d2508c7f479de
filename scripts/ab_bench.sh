# A/B the full bench step of the working tree (A) against a reference tree in ab_old/ (B),
# interleaved ABAB on one box.   bash scripts/ab_bench.sh [bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for it in 1 2; do
  echo "== A round $it"
  timeout -k 10 300 python $R/bench.py --no-cpu-baseline $* 2>&1 | grep '"metric"' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'])" || exit 1
  echo "== B round $it"
  timeout -k 10 300 python $R/ab_old/bench.py --no-cpu-baseline $* 2>&1 | grep '"metric"' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'])" || exit 1
done
