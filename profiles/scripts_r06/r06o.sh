set -o pipefail
cd $GRAFT_REPO_ROOT
for v in "" _ko1 _ko2 _ko3 _w32; do
  DUCOSY_HIP_LIB=$PWD/ducosy-gan_amd/lib/libducosy_hip$v.so timeout -k 10 120 python scripts/kbench.py --only res --mma f16x3 --batch 16 --reps 30 > gpurun_out/r06o_kb$v.log 2>&1 || exit 1
done
