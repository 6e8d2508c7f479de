set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_win.py > gpurun_out/r06n_win.log 2>&1 || { echo TESTFAIL; exit 1; }
timeout -k 10 120 python scripts/kbench.py --only res --mma f16x3 --batch 16 --reps 20 > gpurun_out/r06n_kb16.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r06n_bench16.log 2>&1 || exit 1
DUCOSY_HIP_LIB=$PWD/ducosy-gan_amd/lib/libducosy_hip_w32.so timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r06n_bench32.log 2>&1 || exit 1
bash scripts/pmc_stall.sh r06n16 --only res --mma f16x3 --batch 16
