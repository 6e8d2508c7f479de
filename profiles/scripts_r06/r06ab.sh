# config 5: every phase-kernel layer on fp16 operands in the fp16 mode (candidate default) vs the f16x3 set
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
OLD="up1,up2,pg64,pg128,pg256"
timeout -k 10 900 python -u -m pytest -q -x --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_gpu_concurrent.py tests/test_gpu_fullsize.py -k "f16" -s > gpurun_out/r06ab_tests.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed|worst|Error" gpurun_out/r06ab_tests.log | head -8
for it in 1 2; do
  timeout -k 10 200 python scripts/diag/bench_phase16.py "" --no-cpu-baseline --mma f16 > gpurun_out/r06ab_f16_new_$it.log 2>&1 || exit 1
  echo "new/$it: $(tail -1 gpurun_out/r06ab_f16_new_$it.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')"
  timeout -k 10 200 python scripts/diag/bench_phase16.py "$OLD" --no-cpu-baseline --mma f16 > gpurun_out/r06ab_f16_old_$it.log 2>&1 || exit 1
  echo "old/$it: $(tail -1 gpurun_out/r06ab_f16_old_$it.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')"
done
