# Full-step bench in the three MFMA operand modes (one JSON line each).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for m in ${MODES:-f32 bf16x6 bf16x3 bf16}; do
  timeout -k 10 400 python bench.py --mma $m --no-cpu-baseline > gpurun_out/bm_$m.log 2>&1 || { echo "bench $m failed"; tail -20 gpurun_out/bm_$m.log; exit 1; }
  grep -h '^{' gpurun_out/bm_$m.log
done
