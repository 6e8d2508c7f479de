# Per-layer kernel times of the MFMA convolutions in the exact-f32 and bf16x6 modes (bs 8).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for m in f32 bf16x6; do
  timeout -k 10 200 python scripts/kbench.py --mma $m --only down1,down2,res,up1,up2,d1,d2,d3 > gpurun_out/kball_$m.log 2>&1 || { tail -20 gpurun_out/kball_$m.log; exit 1; }
done
paste gpurun_out/kball_f32.log gpurun_out/kball_bf16x6.log | grep -v amdgpu
