set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
L=$R/ducosy-gan_amd/lib
for v in base sync; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  echo "== $v"; DUCOSY_HIP_LIB=$lib timeout -k 10 200 python -u scripts/diag/win_async_check.py 2>&1 | grep -v amdgpu.ids || exit 1
done
