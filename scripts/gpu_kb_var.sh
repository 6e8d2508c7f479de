# Per-layer kbench of the default library and a VARIANT build side by side, per MMA mode.
#   bash scripts/gpu_kb_var.sh VARIANT "res,down2" "bf16 bf16x3"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
VAR=${1:-buf}
ONLY=${2:-res,down2,d2,d3}
MODES=${3:-bf16 bf16x3}
for m in $MODES; do
  timeout -k 10 200 python scripts/kbench.py --mma $m --only $ONLY > gpurun_out/kv_base_$m.log 2>&1 || { echo "kbench base $m failed"; tail -20 gpurun_out/kv_base_$m.log; exit 1; }
  DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$VAR.so timeout -k 10 200 python scripts/kbench.py --mma $m --only $ONLY > gpurun_out/kv_${VAR}_$m.log 2>&1 || { echo "kbench $VAR $m failed"; tail -20 gpurun_out/kv_${VAR}_$m.log; exit 1; }
  echo "== mode $m: base | $VAR"
  paste gpurun_out/kv_base_$m.log gpurun_out/kv_${VAR}_$m.log | grep -v amdgpu
done
