set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in full l2p; do
  LIB=$R/ducosy-gan_amd/lib/libducosy_hip.so; [ $v = l2p ] && LIB=$R/ducosy-gan_amd/lib/libducosy_hip_l2p.so
  DUCOSY_HIP_LIB=$LIB DUCOSY_X6P=1 DCS_X6P_VARIANT=3 timeout -k 10 120 python3 $R/scripts/kbench.py --only res --mma bf16x6 --reps 5 > $R/gpurun_out/l2p_$v.log 2>&1 || exit 1
  echo "$v"; grep res $R/gpurun_out/l2p_$v.log | head -2
  DUCOSY_HIP_LIB=$LIB DUCOSY_X6P=1 DCS_X6P_VARIANT=3 timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc_l2p_${v}_1 -o p --output-format csv -- python3 $R/scripts/kbench.py --only res --mma bf16x6 --reps 2 > $R/gpurun_out/pmc_l2p_$v.log 2>&1 || exit 1
done
