set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > gpurun_out/gpu_tests4.log 2>&1; echo "TESTS EXIT $?"
grep -E "passed|failed|FAILED" gpurun_out/gpu_tests4.log | tail -8
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "SMOKE EXIT $?"; tail -3 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench1.log 2>&1; echo "BENCH EXIT $?"; tail -5 gpurun_out/bench1.log
