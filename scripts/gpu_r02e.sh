# tests of the touched paths, then the profile set of the bench step at HEAD (tag r02c)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_train.py tests/test_gpu_fullsize.py > gpurun_out/e_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/e_tests.log | head -20; exit 1; }
tail -1 gpurun_out/e_tests.log
bash scripts/gpu_prof_r02.sh r02c || exit 1
