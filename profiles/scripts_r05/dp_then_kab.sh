# the DP product-step tests, then the kernel-variant A/B (scripts/r05/kab.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1; shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp_step.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_dp.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|^E " gpurun_out/${T}_dp.log | head -30; tail -1 gpurun_out/${T}_dp.log
[ $rc -le 1 ] || exit 1
bash scripts/r05/kab.sh $T "$@"
