set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for m in bf16x3 bf16x6 f32; do echo "== $m"; timeout -k 10 400 python scripts/dbg/nan_guard_probe.py $m > gpurun_out/ng_$m.log 2>&1 || { tail -5 gpurun_out/ng_$m.log; exit 1; }; grep -c GUARD gpurun_out/ng_$m.log; grep GUARD gpurun_out/ng_$m.log | sort | uniq -c | sort -rn | head -20; tail -3 gpurun_out/ng_$m.log; done
