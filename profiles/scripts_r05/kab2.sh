# kab.sh, then a short bench per variant (interleaved): bash scripts/r05/kab2.sh TAG VARIANT...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1
bash scripts/r05/kab.sh "$@" || exit 1
shift
L=$R/ducosy-gan_amd/lib
for v in "$@"; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_bench_$v.log 2>&1 || { echo "BENCH $v FAILED"; tail -3 gpurun_out/${T}_bench_$v.log; exit 1; }
  echo "bench $v: $(tail -1 gpurun_out/${T}_bench_$v.log | cut -c1-140)"
done
