# regression at the final code: full GPU suite, smoke, default and f16 benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T=r06ar
timeout -k 10 900 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests -p no:cacheprovider > gpurun_out/${T}_gpu.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/${T}_gpu.log
grep -E "^FAILED" gpurun_out/${T}_gpu.log | head
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKEFAIL; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 1
echo "bench: $(tail -1 gpurun_out/${T}_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["cpu_baseline"]["value"], d["finite"])')"
timeout -k 10 200 python bench.py --no-cpu-baseline --mma f16 > gpurun_out/${T}_bench_f16.log 2>&1 || exit 1
echo "f16: $(tail -1 gpurun_out/${T}_bench_f16.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["finite"])')"
