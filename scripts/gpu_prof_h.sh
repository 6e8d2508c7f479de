set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/profile.sh r01h || exit 1
cd $R
timeout -k 10 300 python scripts/kbench.py > gpurun_out/kbench_r01h.log 2>&1 || { echo "kbench failed"; tail -20 gpurun_out/kbench_r01h.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_masks -o masks --output-format csv -- python3 $R/scripts/bench_masks.py --kinds lung,mediastinum,bone,lung_vessel > $R/gpurun_out/prof_masks.log 2>&1 || { echo "mask prof failed"; exit 1; }
echo all ok
