# core clock of the residual weight gradient in the bench step and the bench value for probe
# libraries:  bash scripts/r05/clk_ab.sh TAG VARIANT...   (each VARIANT a -DCLK_PROBE=1 build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1; shift
for it in 1 2; do
for v in "$@"; do
  DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$v.so timeout -k 10 300 python -u scripts/r05/clk_probe.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/${T}_${v}_${it}.log 2>&1 || { echo "$v FAILED"; tail -3 gpurun_out/${T}_${v}_${it}.log; exit 1; }
  echo "$v/$it: $(grep -o '"value": [0-9.]*' gpurun_out/${T}_${v}_${it}.log) $(grep 'core clock' gpurun_out/${T}_${v}_${it}.log)"
done
done
