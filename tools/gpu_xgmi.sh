#!/bin/bash
# xGMI all-reduce rehearsal: 2 ranks on the box's GPU (gloo for reference collectives).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621 \
  tools/xgmi_check.py --backend gloo > gpurun_out/xgmi_check.log 2>&1 || { echo "xgmi_check failed"; tail -60 gpurun_out/xgmi_check.log; exit 1; }
grep '^{' gpurun_out/xgmi_check.log
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29622 \
  bench.py --gpus 2 --backend gloo --allreduce xgmi --steps 400 --warmup 40 > gpurun_out/xgmi_bench.log 2>&1 || { echo "xgmi bench failed"; tail -40 gpurun_out/xgmi_bench.log; exit 1; }
tail -1 gpurun_out/xgmi_bench.log
