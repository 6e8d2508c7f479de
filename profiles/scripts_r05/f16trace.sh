# kernel trace of the f16-mode bench step (BASELINE config 5's operand mode)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${T}_f16tr -o tr -- python3 $R/bench.py --mma f16 --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_f16tr.log 2>&1 || exit 1
tail -1 $R/gpurun_out/${T}_f16tr.log | cut -c1-150
