# stall counters of the window phase kernels (up-convs: forward MODE 0, data gradient MODE 1; down1) at
# HEAD, then the default and f16 bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/pmc_stall.sh r05h --only up1,down1 --mma f16x3 --batch 16 || exit 1
cd $R && timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r05h_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r05h_bench.log | cut -c1-200
timeout -k 10 300 python -u bench.py --mma f16 --no-cpu-baseline > gpurun_out/r05h_bench_f16.log 2>&1 || exit 1
tail -1 gpurun_out/r05h_bench_f16.log | cut -c1-200
