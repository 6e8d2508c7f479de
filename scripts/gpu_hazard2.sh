# Two-stream hazard probes (Config 5).  Each probe runs fresh systems and compares
# with the sequential run; none is part of the product path.
#   bash scripts/gpu_hazard2.sh [MODE]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
M=${1:-bf16x6}
cd $R && mkdir -p gpurun_out
echo "== overlap vs stream identity (a: overlapping, b: synced per model, c: one side stream)"
timeout -k 10 400 python scripts/conc_diag4.py $M 8 || exit 1
echo "== unrelated co-runner (x6 weight gradient) beside one model"
timeout -k 10 300 python scripts/conc_noise.py $M 6 wgrad 300 || exit 1
echo "== first differing op (conv passes and packs traced)"
TRACE_ONLY=conv timeout -k 10 400 python scripts/conc_trace2.py $M 10 || exit 1
echo "== every op replayed under a co-runner"
timeout -k 10 400 python scripts/race_hunt.py $M 12 || exit 1
echo "== pool poisoning (reads of never-written memory)"
timeout -k 10 300 python scripts/uninit_probe.py $M || exit 1
echo "== NaN guard allocator (out-of-bounds reads / writes)"
timeout -k 10 400 python scripts/dbg/nan_guard_probe.py $M || exit 1
