set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/r06r_gpu.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06r_smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r06r_bench.log 2>&1 || exit 1
DUCOSY_HIP_LIB=$PWD/ducosy-gan_amd/lib/libducosy_hip_w32.so timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r06r_bench32.log 2>&1 || exit 1
