# A/B/C... per-layer kernel timings of several library builds on one box, interleaved by round.
#   bash scripts/ab_multi.sh "v1 v2 ..." "kbench args"   (variant "def" = lib/libducosy_hip.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
VS=$1; shift
ARGS="$*"
mkdir -p $R/gpurun_out
for it in 1 2 3; do
  for v in $VS; do
    if [ "$v" = def ]; then lib=libducosy_hip.so; else lib=libducosy_hip_$v.so; fi
    echo "== $v (round $it)"
    DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/$lib timeout -k 10 200 python $R/scripts/kbench.py $ARGS 2>&1 | grep -v -e amdgpu.ids -e '^layer' || exit 1
  done
done
