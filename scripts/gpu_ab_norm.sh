# parity tests then whole-step A/B against lib/libducosy_hip_$1.so
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/q_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/q_tests.log | head -20; exit 1; }
tail -1 gpurun_out/q_tests.log
bash scripts/ab_lib.sh $1 || exit 1
