# at a committed HEAD: full GPU suite, then the kernel table's rocprofv3 passes (trace, FETCH_SIZE, WRITE_SIZE, MFMA busy)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=${1:-r04u}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_full_tests.log 2>&1
rc=$?
grep -E "FAILED|^E  " gpurun_out/${T}_full_tests.log | head -20; tail -1 gpurun_out/${T}_full_tests.log
[ $rc -le 1 ] || exit 1
bash scripts/gpu_prof_r02.sh $T || exit 1
echo done
