set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/diag/bign_stages.py 48 > gpurun_out/r06f_stages.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_win.py tests/test_gpu_fullsize.py > gpurun_out/r06f_win.log 2>&1 || { echo TESTFAIL; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r06f_bench16.log 2>&1 || exit 1
DUCOSY_HIP_LIB=$PWD/ducosy-gan_amd/lib/libducosy_hip_w32.so timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r06f_bench32.log 2>&1 || exit 1
