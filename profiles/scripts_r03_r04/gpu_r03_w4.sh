# one-wave-per-SIMD window forward (variant w4): window / ops tests on it, kbench res A/B x2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V=${1:-w4}
DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_win.py tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/w4_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|^E  " gpurun_out/w4_tests.log | head -20; tail -3 gpurun_out/w4_tests.log; exit 1; }
tail -1 gpurun_out/w4_tests.log
bash scripts/gpu_kab.sh res f16x3 16 $V || exit 1
bash scripts/gpu_kab.sh res f16x3 16 $V || exit 1
