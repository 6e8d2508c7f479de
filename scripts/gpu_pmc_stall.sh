# Stall breakdown (SQ counters) of the residual-conv kernels: two PMC passes over kbench res.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python3 $R/scripts/kbench.py --only res --mma bf16x6 --batch 16 --reps 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d $R/gpurun_out/pmc_st1 -o p --output-format csv -- $B > $R/gpurun_out/pmc_st1.log 2>&1 || exit 1
echo pass1 ok
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_st2 -o p --output-format csv -- $B > $R/gpurun_out/pmc_st2.log 2>&1 || exit 1
echo pass2 ok
