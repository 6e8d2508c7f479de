# PMC counters for one layer's kernels (kbench), separate rocprofv3 passes.
#   bash scripts/pmc_res.sh TAG "kbench args"     e.g.  bash scripts/pmc_res.sh r01d "--only res --nopro"
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-res}; shift
ARGS=${*:---only res}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc_${TAG}_$i -o p --output-format csv \
    -- python3 $R/scripts/kbench.py $ARGS --reps 2 > $R/gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo pmc done
