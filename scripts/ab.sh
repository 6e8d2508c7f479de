# A/B per-layer kernel timings of two library builds on the same box, interleaved ABAB.
#   bash scripts/ab.sh VARIANT "kbench args"      (A = lib/libducosy_hip.so, B = lib/libducosy_hip_VARIANT.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=$1; shift
ARGS="$*"
mkdir -p $R/gpurun_out
for it in 1 2; do
  for lib in libducosy_hip.so libducosy_hip_$V.so; do
    echo "== $lib (round $it)"
    DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/$lib timeout -k 10 200 python $R/scripts/kbench.py $ARGS 2>&1 | grep -v -e amdgpu.ids -e '^layer' || exit 1
  done
done
