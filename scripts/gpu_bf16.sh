# half-precision (config 5) path: bf16 bench lines (one model, both models) and the bf16 kernel profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --mma bf16 > gpurun_out/bf16_bench.log 2>&1 || { echo BENCH FAILED; tail -3 gpurun_out/bf16_bench.log; exit 1; }
echo "bf16: $(tail -1 gpurun_out/bf16_bench.log | cut -c60-120)"
timeout -k 10 300 python bench.py --no-cpu-baseline --dual --mma bf16 > gpurun_out/bf16_dual_bench.log 2>&1 || { echo BENCH FAILED; tail -3 gpurun_out/bf16_dual_bench.log; exit 1; }
echo "bf16 dual: $(tail -1 gpurun_out/bf16_dual_bench.log | cut -c60-120)"
timeout -k 10 300 python bench.py --no-cpu-baseline --dual --dual-schedule concurrent --mma bf16 > gpurun_out/bf16_dualc_bench.log 2>&1 || { echo BENCH FAILED; tail -3 gpurun_out/bf16_dualc_bench.log; exit 1; }
echo "bf16 dual concurrent: $(tail -1 gpurun_out/bf16_dualc_bench.log | cut -c60-120)"
BENCH_EXTRA="--mma bf16" bash scripts/gpu_prof_r02.sh ${1:-r02g_bf16}
