# kbench A/B of library variants at the production shapes: default library, then each variant
#   bash scripts/gpu_kab.sh "LAYERS" MODE BATCH VARIANT...    (LAYERS: kbench --only list, "" = all)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
ONLY=$1; MODE=$2; BATCH=$3; shift 3
timeout -k 10 300 python scripts/kbench.py --batch $BATCH --reps 5 --mma $MODE --only "$ONLY" > gpurun_out/kab_A.log 2>&1 || { echo KBENCH A FAILED; tail -5 gpurun_out/kab_A.log; exit 1; }
echo "== A (default)"; grep -v amdgpu.ids gpurun_out/kab_A.log
for V in "$@"; do
  DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$V.so timeout -k 10 300 python scripts/kbench.py --batch $BATCH --reps 5 --mma $MODE --only "$ONLY" > gpurun_out/kab_$V.log 2>&1 || { echo KBENCH $V FAILED; tail -5 gpurun_out/kab_$V.log; exit 1; }
  echo "== $V"; grep -v amdgpu.ids gpurun_out/kab_$V.log
done
