# window kernel v2 (conv3_win2_kernel): window tests, then kbench res A/B against v1 (DCS_WIN_V1=1)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04c}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_win.py > gpurun_out/${T}_win_tests.log 2>&1 || { echo WIN TESTS FAILED; grep -E "FAILED|Error|^E  " gpurun_out/${T}_win_tests.log | head -20; exit 1; }
tail -1 gpurun_out/${T}_win_tests.log
for i in 1 2; do
  DCS_WIN_V1=1 timeout -k 10 120 python scripts/kbench.py --only res --mma f16x3 --batch 16 --reps 9 > gpurun_out/${T}_kb_v1_$i.log 2>&1 || exit 1
  timeout -k 10 120 python scripts/kbench.py --only res --mma f16x3 --batch 16 --reps 9 > gpurun_out/${T}_kb_v2_$i.log 2>&1 || exit 1
done
grep -h "res" gpurun_out/${T}_kb_v*_*.log
