# Two-stream hazard: a build without scalarised device-data loads, with kernel arguments in device
# memory (HIP_FORCE_DEV_KERNARG=1) and in host memory (=0); shared CUs (variant t)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
L=$R/ducosy-gan_amd/lib/libducosy_hip_nosl.so
for ka in 1 0; do
  DUCOSY_HIP_LIB=$L HIP_FORCE_DEV_KERNARG=$ka timeout -k 10 400 python -u scripts/conc_cumask.py bf16x6 ${1:-24} t > gpurun_out/kernarg_$ka.log 2>&1 || { echo PROBE FAILED; tail -3 gpurun_out/kernarg_$ka.log; exit 1; }
  echo "nosl, HIP_FORCE_DEV_KERNARG=$ka: $(tail -1 gpurun_out/kernarg_$ka.log)"
done
timeout -k 10 400 python -u scripts/conc_cumask.py bf16x6 ${1:-24} t > gpurun_out/kernarg_default.log 2>&1 || exit 1
echo "default build: $(tail -1 gpurun_out/kernarg_default.log)"
