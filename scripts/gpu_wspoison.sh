set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python scripts/ws_poison.py bf16x6 bf16x3 f32 > gpurun_out/wsp0.json 2>/dev/null || exit 1
DUCOSY_WS_POISON=1 timeout -k 10 300 python scripts/ws_poison.py bf16x6 bf16x3 f32 > gpurun_out/wsp1.json 2>/dev/null || exit 1
python - <<'PY'
import json
a = json.load(open("gpurun_out/wsp0.json")); b = json.load(open("gpurun_out/wsp1.json"))
for k in a:
    print(k, "identical" if a[k] == b[k] else "DIFFER", [ (i, x["loss_G"], y["loss_G"]) for i, (x, y) in enumerate(zip(a[k], b[k])) if x != y][:3])
PY
