# full GPU suite, smoke, bench; config-5 schedules (serial, concurrent on CU-partitioned streams)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/gpu_full.sh || exit 1
for sch in serial concurrent; do
  timeout -k 10 400 python bench.py --dual --dual-schedule $sch --no-cpu-baseline > gpurun_out/dual_$sch.log 2>&1 || { echo DUAL FAILED; tail -3 gpurun_out/dual_$sch.log; exit 1; }
  echo "dual $sch: $(tail -1 gpurun_out/dual_$sch.log | cut -c1-140)"
done
