# phase-kernel tests on the default library, then kbench of the phase-kernel layers (and res), default vs
# variants, interleaved:  bash scripts/r05/sp_ab.sh TAG VARIANT...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_subpix.py tests/test_gpu_win.py tests/test_gpu_train.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_tests.log | head -10; tail -1 gpurun_out/${T}_tests.log
[ $rc -le 1 ] || exit 1
SKIP_TESTS=1 KB_ONLY=${KB_ONLY:-res,up1,up2,down1,down2,d1,d2,d3} bash scripts/r05/full_ab.sh "$@"
