# config 5: which phase-kernel layers hold the f16 fixture bar on fp16 operands
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/diag/f16_layers.py > gpurun_out/r06aa_f16_layers.log 2>&1; echo "rc=$?"; cat gpurun_out/r06aa_f16_layers.log | grep -v amdgpu.ids
