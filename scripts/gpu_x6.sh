# bf16x6 check: MMA mode tests, per-layer kernels, and the full step in f32 / bf16x6.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/gpu_mma.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q -k mma_modes --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/x6_train.log 2>&1 || { echo "TRAIN TESTS FAILED"; tail -40 gpurun_out/x6_train.log; exit 1; }
tail -2 gpurun_out/x6_train.log
MODES="bf16x6 f32" bash scripts/gpu_bench_modes.sh
