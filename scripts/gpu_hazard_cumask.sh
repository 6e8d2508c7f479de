# Two-stream hazard localisation (Config 5): fresh two-model concurrent runs against
# the sequential run, with the two streams on shared / disjoint / interleaved compute units.
#   bash scripts/gpu_hazard_cumask.sh [ATTEMPTS] [VARIANTS]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/conc_cumask.py bf16x6 ${1:-20} ${2:-t,m,g,e} > gpurun_out/cumask.log 2>&1 || { echo PROBE FAILED; tail -5 gpurun_out/cumask.log; exit 1; }
tail -6 gpurun_out/cumask.log
