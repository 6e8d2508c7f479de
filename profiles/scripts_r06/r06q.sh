set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_win.py > gpurun_out/r06q_win.log 2>&1 || { echo TESTFAIL; exit 1; }
for rep in 1 2; do
for v in "" _wg32 _v1 _v2 _w32; do
  DUCOSY_HIP_LIB=$PWD/ducosy-gan_amd/lib/libducosy_hip$v.so timeout -k 10 120 python scripts/kbench.py --only res --mma f16x3 --batch 16 --reps 40 > gpurun_out/r06q_kb${v}_$rep.log 2>&1 || exit 1
done
done
for v in "" _wg32 _v1 _v2 _w32; do
  DUCOSY_HIP_LIB=$PWD/ducosy-gan_amd/lib/libducosy_hip$v.so timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r06q_bench$v.log 2>&1 || exit 1
done
