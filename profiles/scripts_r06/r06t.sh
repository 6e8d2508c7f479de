set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -q -x --timeout 600 --timeout-method thread -m gpu tests -k "not config4" > gpurun_out/r06t_gpu.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r06t_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r06t_bench.log 2>&1 || exit 1
