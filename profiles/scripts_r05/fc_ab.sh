# residual window conv fixed-cost probe (scripts/r05/fixed_cost.py, f16x3) for the default and variant
# libraries, then both_ab.sh's bench-step traces:  bash scripts/r05/fc_ab.sh TAG VARIANT...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1; shift
L=$R/ducosy-gan_amd/lib
for v in base "$@"; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 300 python -u scripts/r05/fixed_cost.py --mma f16x3 > gpurun_out/${T}_fc_$v.log 2>&1 || { echo "FC $v FAILED"; tail -3 gpurun_out/${T}_fc_$v.log; exit 1; }
  echo "$v: $(grep -E '^cin  256|^fwd' gpurun_out/${T}_fc_$v.log | tr '\n' ' ')"
done
bash scripts/r05/both_ab.sh $T "$@"
