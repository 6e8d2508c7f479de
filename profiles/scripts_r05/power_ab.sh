# power / clock telemetry around the bench step for probe libraries (read-only rocm-smi / amd-smi
# queries):  bash scripts/r05/power_ab.sh TAG VARIANT...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1; shift
for v in "$@"; do
  timeout -k 5 60 amd-smi metric > gpurun_out/${T}_${v}_smi_before.txt 2>&1
  ( for i in $(seq 1 120); do date +%s.%N; timeout -k 2 10 rocm-smi -P -c -t --csv 2>/dev/null; sleep 0.25; done ) > gpurun_out/${T}_${v}_samples.txt 2>&1 &
  SP=$!
  DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$v.so timeout -k 10 300 python -u scripts/r05/clk_probe.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_${v}.log 2>&1
  rc=$?
  kill $SP 2>/dev/null; wait $SP 2>/dev/null
  timeout -k 5 60 amd-smi metric > gpurun_out/${T}_${v}_smi_after.txt 2>&1
  [ $rc -eq 0 ] || { echo "$v FAILED"; tail -3 gpurun_out/${T}_${v}.log; exit 1; }
  echo "$v: $(grep -o '"value": [0-9.]*' gpurun_out/${T}_${v}.log) $(grep 'core clock' gpurun_out/${T}_${v}.log)"
  sleep 20
done
