# stall breakdown (SQ / LDS / MFMA counters) of the f16x3 up-conv phase kernels and the f16 residual
# weight gradient, for the next round's analysis
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/pmc_stall.sh r06ao_up --only up1,up2 --batch 8 || exit 1
bash scripts/pmc_stall.sh r06ao_resh --only res --mma f16 --batch 16 || exit 1
bash scripts/pmc_stall.sh r06ao_res --only res --batch 16 || exit 1
cd $R
for t in r06ao_up r06ao_resh r06ao_res; do python scripts/pmc_table.py $t _kernel > gpurun_out/${t}_table.txt 2>&1; done
rm -rf gpurun_out/pmc_r06ao_*_[0-9]
cat gpurun_out/r06ao_up_table.txt | head -30
