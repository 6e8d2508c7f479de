# pmc stall passes of the residual window kernels, new (16x16x32) and old (32x32x16) library
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python scripts/kbench.py --only res --mma f16x3 --batch 16 --reps 20 > gpurun_out/r06h_kb16.log 2>&1 || exit 1
DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_w32.so timeout -k 10 120 python scripts/kbench.py --only res --mma f16x3 --batch 16 --reps 20 > gpurun_out/r06h_kb32.log 2>&1 || exit 1
bash scripts/pmc_stall.sh r06h16 --only res --mma f16x3 --batch 16 || exit 1
DUCOSY_HIP_LIB=$R/ducosy-gan_amd/lib/libducosy_hip_w32.so bash scripts/pmc_stall.sh r06h32 --only res --mma f16x3 --batch 16 || exit 1
