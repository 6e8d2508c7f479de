# window-kernel bring-up: its tests, the op / MMA tests, kbench of the residual layer, one bench line
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_ops.py tests/test_gpu_mma.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/win_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/win_tests.log | head -30; exit 1; }
tail -1 gpurun_out/win_tests.log
timeout -k 10 200 python scripts/kbench.py --batch 16 --reps 5 --mma f16x3 --only res > gpurun_out/kbench_win.log 2>&1 || { echo KBENCH FAILED; tail -5 gpurun_out/kbench_win.log; exit 1; }
cat gpurun_out/kbench_win.log | grep res
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bench_win.log 2>&1 || { echo BENCH FAILED; tail -5 gpurun_out/bench_win.log; exit 1; }
tail -1 gpurun_out/bench_win.log | cut -c1-220
