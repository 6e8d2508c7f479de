set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_masks.py tests/test_gpu_dataset.py tests/test_gpu_models.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/d_tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/d_tests.log; exit 1; }
tail -4 gpurun_out/d_tests.log
