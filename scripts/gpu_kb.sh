set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
ONLY=${1:-res,down2,d2,d3}
for m in f32 bf16 bf16x3 bf16x6; do
  timeout -k 10 200 python scripts/kbench.py --mma $m --only $ONLY > gpurun_out/kb_$m.log 2>&1 || { echo "kbench $m failed"; tail -20 gpurun_out/kb_$m.log; exit 1; }
done
paste gpurun_out/kb_f32.log gpurun_out/kb_bf16.log gpurun_out/kb_bf16x3.log | grep -v amdgpu
