# full GPU suite at the ring16 / staging commit, smoke, default bench, f16 (config 5) bench vs the rows-pass ring
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
L=$R/ducosy-gan_amd/lib
timeout -k 10 900 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests -p no:cacheprovider > gpurun_out/r06x_gpu.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/r06x_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06x_smoke.log 2>&1 || { echo SMOKEFAIL; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r06x_bench.log 2>&1 || exit 1
echo "bench: $(tail -1 gpurun_out/r06x_bench.log | cut -c80-125)"
for v in base r0; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --mma f16 > gpurun_out/r06x_bench_f16_$v.log 2>&1 || exit 1
  echo "f16 $v: $(tail -1 gpurun_out/r06x_bench_f16_$v.log | cut -c80-125)"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --mma f16 --dual > gpurun_out/r06x_bench_dual_f16.log 2>&1 || exit 1
echo "dual f16: $(tail -1 gpurun_out/r06x_bench_dual_f16.log | cut -c80-125)"
