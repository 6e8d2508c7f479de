# smoke of the other bench modes at HEAD: fp16 / bf16x6 / f32 operand modes, config-5 dual (serial, concurrent), G_A2B workload
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for args in "--mma f16" "--mma bf16x6" "--mma f32 --steps 2 --warmup 1" "--dual --steps 3 --warmup 1" "--dual --dual-schedule concurrent --steps 3 --warmup 1" "--workload g_a2b --steps 3 --warmup 1" "--mma bf16 --steps 3 --warmup 1"; do
  tag=$(echo "$args" | tr -d ' -' | cut -c1-30)
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > gpurun_out/m_$tag.log 2>&1 || { echo "BENCH $args FAILED"; tail -5 gpurun_out/m_$tag.log; exit 1; }
  echo "$args: $(tail -1 gpurun_out/m_$tag.log | cut -c1-230)"
done
