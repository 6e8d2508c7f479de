# Stall breakdown of one layer's kernels (kbench): SQ issue/wait/active cycles, LDS and MFMA
# counters, in separate rocprofv3 passes (<= 8 SQ counters each).
#   bash scripts/pmc_stall.sh TAG "kbench args"
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-stall}; shift
ARGS=${*:---only res --mma bf16x6 --batch 16}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INST_CYCLES_VMEM_RD SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc_${TAG}_$i -o p --output-format csv \
    -- python3 $R/scripts/kbench.py $ARGS --reps 2 > $R/gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo pmc done
