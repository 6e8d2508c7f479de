# prologue A/B: window-conv workgroup phase times (timing probe library), then both_ab.sh's tests and
# bench-step traces, default vs variants:  bash scripts/r05/pro_ab.sh TAG VARIANT...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1; shift
DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_tm.so timeout -k 10 200 python -u scripts/r05/win_timing.py > gpurun_out/${T}_wt.log 2>&1 || { tail -3 gpurun_out/${T}_wt.log; exit 1; }
cat gpurun_out/${T}_wt.log
bash scripts/r05/both_ab.sh $T "$@"
