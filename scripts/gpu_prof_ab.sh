# Kernel-trace stats of a short bench run with the default library and a VARIANT build.
#   bash scripts/gpu_prof_ab.sh VARIANT
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=$1
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_base -o t --output-format csv \
  -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/ab_base.log 2>&1 || exit 1
DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$V.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_$V -o t --output-format csv \
  -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/ab_$V.log 2>&1 || exit 1
echo ab ok
