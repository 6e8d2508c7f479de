# A/B of two library builds on the bench step, interleaved ABAB, plus a kernel-stats trace of each.
#   bash scripts/ab_lib.sh VARIANT      (B = ducosy-gan_amd/lib/libducosy_hip_VARIANT.so)
set -o pipefail
#   BENCH_EXTRA="--mma bf16" benchmarks another operand mode
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=$1
cd $R && mkdir -p gpurun_out
B=$R/ducosy-gan_amd/lib/libducosy_hip_$V.so
for it in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_EXTRA > gpurun_out/ab_A_$it.log 2>&1 || { echo BENCH A FAILED; tail -3 gpurun_out/ab_A_$it.log; exit 1; }
  echo "A default: $(tail -1 gpurun_out/ab_A_$it.log | cut -c80-125)"
  DUCOSY_HIP_LIB=$B timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_EXTRA > gpurun_out/ab_B_$it.log 2>&1 || { echo BENCH B FAILED; tail -3 gpurun_out/ab_B_$it.log; exit 1; }
  echo "B $V: $(tail -1 gpurun_out/ab_B_$it.log | cut -c80-125)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_A_prof -o a --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_EXTRA > $R/gpurun_out/ab_A_prof.log 2>&1 || exit 1
DUCOSY_HIP_LIB=$B timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_B_prof -o b --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_EXTRA > $R/gpurun_out/ab_B_prof.log 2>&1 || exit 1
echo prof ok
