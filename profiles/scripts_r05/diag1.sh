# stall counters of the residual kernels at HEAD, then the config-2 gradient errors against a float64 oracle
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/pmc_stall.sh r05g --only res --mma f16x3 --batch 16 || exit 1
cd $R && timeout -k 10 900 python -u scripts/diag/oracle_f64_floor.py f32 f16x3 > gpurun_out/r05g_f64floor.log 2>&1 || { tail -5 gpurun_out/r05g_f64floor.log; exit 1; }
tail -4 gpurun_out/r05g_f64floor.log
