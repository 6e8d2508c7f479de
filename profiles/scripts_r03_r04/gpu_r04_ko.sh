# knock-out timing probes of conv3_win2_kernel (results wrong by design): kbench res fwd, f16x3, bs 16
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04i}
for ko in ${KOS:-0 1 2 4 3 6 7}; do
  DCS_WIN2_KO=$ko timeout -k 10 120 python scripts/kbench.py --only res --mma f16x3 --batch 16 --reps 9 > gpurun_out/${T}_ko$ko.log 2>&1 || exit 1
  echo "ko=$ko $(grep 'res *fwd' gpurun_out/${T}_ko$ko.log)"
done
