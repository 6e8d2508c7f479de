set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dataset.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/ds_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ds_tests.log; exit 1; }
tail -1 gpurun_out/ds_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_masks2 -o masks --output-format csv -- python3 $R/scripts/bench_masks.py --kinds lung,mediastinum,bone,lung_vessel > $R/gpurun_out/prof_masks2.log 2>&1 || { echo "mask prof failed"; exit 1; }
echo prof ok
