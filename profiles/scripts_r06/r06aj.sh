# verification at the round-6 f16 defaults (paired phase-kernel iterations for the forward-type launches,
# stem / head on fp16 operands in the f16 mode): full GPU suite, smoke, benches, f16 A/B against one
# iteration per barrier (p0 lib), then the kernel-table profile passes of the default and f16 steps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r06aj}
L=$R/ducosy-gan_amd/lib
timeout -k 10 900 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests -p no:cacheprovider > gpurun_out/${T}_gpu.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/${T}_gpu.log
grep -E "^FAILED" gpurun_out/${T}_gpu.log | head
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKEFAIL; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 1
echo "bench: $(tail -1 gpurun_out/${T}_bench.log | cut -c80-125)"
for it in 1 2; do
  for v in p0 def; do
    lib=$L/libducosy_hip_$v.so; [ "$v" = def ] && lib=$L/libducosy_hip.so
    DUCOSY_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --mma f16 > gpurun_out/${T}_f16_${v}_$it.log 2>&1 || exit 1
    echo "f16 $v/$it: $(tail -1 gpurun_out/${T}_f16_${v}_$it.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["finite"])')"
  done
done
timeout -k 10 300 python bench.py --no-cpu-baseline --mma f16 --dual > gpurun_out/${T}_bench_dual_f16.log 2>&1 || exit 1
echo "dual f16: $(tail -1 gpurun_out/${T}_bench_dual_f16.log | cut -c80-125)"
timeout -k 10 200 python bench.py --no-cpu-baseline --workload g_a2b > gpurun_out/${T}_bench_g_a2b.log 2>&1 || exit 1
echo "g_a2b: $(tail -1 gpurun_out/${T}_bench_g_a2b.log | cut -c80-125)"
bash scripts/gpu_prof_r02.sh $T || exit 1
BENCH_EXTRA="--mma f16" bash scripts/gpu_prof_r02.sh ${T}h || exit 1
