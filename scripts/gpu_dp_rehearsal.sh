# Multi-process rehearsal of the N>1 bench path on ONE GPU (two ranks share cuda:0 over gloo; RCCL
# does not allow two ranks on one device): barrier, MAX-over-ranks timing, bucketed G all-reduce,
# whole-batch loss statistics; then the split-groups config-5 schedule with one rank per group.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export DUCOSY_DIST_BACKEND=gloo DUCOSY_DEVICE_OVERRIDE=0
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dp2.log 2>&1 || { echo DP2 FAILED; tail -5 gpurun_out/dp2.log; exit 1; }
grep '^{' gpurun_out/dp2.log | cut -c1-200
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --dual --dual-schedule groups > gpurun_out/dp2_groups.log 2>&1 || { echo GROUPS FAILED; tail -5 gpurun_out/dp2_groups.log; exit 1; }
grep '^{' gpurun_out/dp2_groups.log | cut -c1-200
