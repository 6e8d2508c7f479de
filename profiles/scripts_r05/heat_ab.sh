# does the persistent window conv's step gain depend on the GPU's thermal state?  bench (default
# library) and bench (VARIANT) on a cold GPU, then the GPU test suite (~2 min), then both again, with
# rocm-smi power / clock / temperature samples:  bash scripts/r05/heat_ab.sh TAG VARIANT
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1; V=$2
L=$R/ducosy-gan_amd/lib
run() {  # run NAME LIB
  ( for i in $(seq 1 100); do date +%s.%N; timeout -k 2 10 rocm-smi -P -c -t --csv 2>/dev/null; sleep 0.25; done ) > gpurun_out/${T}_$1_samples.txt 2>&1 &
  SP=$!
  DUCOSY_HIP_LIB=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_$1.log 2>&1
  rc=$?
  kill $SP 2>/dev/null; wait $SP 2>/dev/null
  [ $rc -eq 0 ] || { echo "$1 FAILED"; tail -3 gpurun_out/${T}_$1.log; exit 1; }
  echo "$1: $(tail -1 gpurun_out/${T}_$1.log | grep -o '"value": [0-9.]*') $(grep '^card0' gpurun_out/${T}_$1_samples.txt | awk -F, '{gsub(/[()Mhz]/,"",$8); if ($12>400) {n++; p+=$12; c+=$8; t=$2}} END {if (n) printf "power %.0f W sclk %.0f MHz T %s C (%d samples)", p/n, c/n, t, n}')"
}
run cold_pers $L/libducosy_hip.so
run cold_$V $L/libducosy_hip_$V.so
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
tail -1 gpurun_out/${T}_tests.log
run hot_pers $L/libducosy_hip.so
run hot_$V $L/libducosy_hip_$V.so
run hot2_pers $L/libducosy_hip.so
