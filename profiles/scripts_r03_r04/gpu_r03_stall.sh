# kbench of every layer (f16x3, bf16x6) and the stall breakdown of the f16x3 residual kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for m in f16x3 bf16x6; do
  timeout -k 10 300 python scripts/kbench.py --batch 16 --reps 5 --mma $m > gpurun_out/kbench_$m.log 2>&1 || { echo KBENCH $m FAILED; tail -5 gpurun_out/kbench_$m.log; exit 1; }
done
bash scripts/pmc_stall.sh h3res --only res --mma f16x3 --batch 16 || exit 1
