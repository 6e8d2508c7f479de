# Skeleton probes of the pre-split residual conv (timing only): full / no DMA / no DMA+barrier /
# no DMA+barrier+LDS reads; MFMA-busy and wave-state counters in one PMC pass each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in full nodma nobar nolds old; do
  LIB=$R/ducosy-gan_amd/lib/libducosy_hip_$v.so; X=1
  [ $v = full ] && LIB=$R/ducosy-gan_amd/lib/libducosy_hip.so
  [ $v = old ] && { LIB=$R/ducosy-gan_amd/lib/libducosy_hip.so; X=0; }
  DUCOSY_HIP_LIB=$LIB DUCOSY_X6P=$X DCS_X6P_VARIANT=3 timeout -k 10 120 python3 $R/scripts/kbench.py --only res --mma bf16x6 --reps 5 > $R/gpurun_out/skel_$v.log 2>&1 || exit 1
  echo "$v"; grep res $R/gpurun_out/skel_$v.log | head -2
  DUCOSY_HIP_LIB=$LIB DUCOSY_X6P=$X DCS_X6P_VARIANT=3 timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_skel_${v}_1 -o p --output-format csv -- python3 $R/scripts/kbench.py --only res --mma bf16x6 --reps 2 > $R/gpurun_out/pmc_skel_$v.log 2>&1 || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r02_step_trace -o k --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/r02_step_trace.log 2>&1 || exit 1
echo trace ok
