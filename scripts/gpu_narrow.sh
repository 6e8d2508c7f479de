set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/nr_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/nr_tests.log; exit 1; }
tail -1 gpurun_out/nr_tests.log
bash scripts/gpu_kb_var.sh ${1:-v1} head,stem,d0 f32
