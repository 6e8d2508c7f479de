# Per-layer kbench of the default library and two variant builds, one MMA mode.
#   bash scripts/gpu_kb_var2.sh VAR1 VAR2 "res,down2" bf16x6
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V1=$1; V2=$2; ONLY=${3:-res}; M=${4:-bf16x6}
timeout -k 10 200 python scripts/kbench.py --mma $M --only $ONLY > gpurun_out/k3_base.log 2>&1 || { tail -20 gpurun_out/k3_base.log; exit 1; }
for v in $V1 $V2; do
  DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$v.so timeout -k 10 200 python scripts/kbench.py --mma $M --only $ONLY > gpurun_out/k3_$v.log 2>&1 || { tail -20 gpurun_out/k3_$v.log; exit 1; }
done
echo "== $M: base | $V1 | $V2"
paste gpurun_out/k3_base.log gpurun_out/k3_$V1.log gpurun_out/k3_$V2.log | grep -v amdgpu
