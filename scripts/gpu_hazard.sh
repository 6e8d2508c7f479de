set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 240 python scripts/hazard_probe.py bf16x6 0 1500 > gpurun_out/hz_x6_reuse.json 2> gpurun_out/hz_x6_reuse.err || exit 1
timeout -k 10 240 python scripts/hazard_probe.py bf16x6 1 1500 > gpurun_out/hz_x6_keep.json 2> gpurun_out/hz_x6_keep.err || exit 1
timeout -k 10 240 python scripts/hazard_probe.py f32 0 1500 > gpurun_out/hz_f32_reuse.json 2> gpurun_out/hz_f32_reuse.err || exit 1
cat gpurun_out/hz_*.json | cut -c1-600
