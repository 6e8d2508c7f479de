# CBAM passes: sa_apply16 loads hoisted (base) vs not (nohoist); fused sums pass with 8 pixels per wave (px8), 2048 blocks (b2k)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
L=$R/ducosy-gan_amd/lib
for v in px8; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06af_tests_$v.log 2>&1 || { echo "TESTFAIL $v"; grep -E "^E  |FAILED" gpurun_out/r06af_tests_$v.log | head; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/r06af_tests_$v.log)"
done
cd /tmp && export TMPDIR=/tmp
for it in 1 2; do
for v in base nohoist px8 b2k; do
  lib=$L/libducosy_hip_$v.so; [ "$v" = base ] && lib=$L/libducosy_hip.so
  DUCOSY_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r06af_tr_${v}_$it -o tr -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/r06af_tr_${v}_$it.log 2>&1 || { echo "TRACE $v FAILED"; exit 1; }
done
done
echo traces ok
cd $R && python3 scripts/trace_cmp.py 7 gpurun_out/r06af_tr_base_1 gpurun_out/r06af_tr_nohoist_1 gpurun_out/r06af_tr_px8_1 gpurun_out/r06af_tr_b2k_1 gpurun_out/r06af_tr_base_2 gpurun_out/r06af_tr_nohoist_2 gpurun_out/r06af_tr_px8_2 gpurun_out/r06af_tr_b2k_2 > gpurun_out/r06af_cmp.txt && rm -rf gpurun_out/r06af_tr_*_[12]
