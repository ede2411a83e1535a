#!/bin/bash
# xGMI all-reduce rehearsal: 2 and 4 ranks sharing the box's GPU (gloo for reference collectives).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for W in 2 4; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port $((29620 + W)) \
    tools/xgmi_check.py --backend gloo --bench > gpurun_out/xgmi_check_w$W.log 2>&1 || { echo "xgmi_check W=$W failed"; tail -60 gpurun_out/xgmi_check_w$W.log; exit 1; }
  grep '^{' gpurun_out/xgmi_check_w$W.log
done
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29630 \
  bench.py --gpus 2 --backend gloo --allreduce xgmi --steps 400 --warmup 40 > gpurun_out/xgmi_bench.log 2>&1 || { echo "xgmi bench failed"; tail -40 gpurun_out/xgmi_bench.log; exit 1; }
tail -1 gpurun_out/xgmi_bench.log
