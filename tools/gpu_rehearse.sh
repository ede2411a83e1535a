#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box (gloo ranks sharing GPU 0) + job latency on MI355X.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --backend gloo --steps 200 --warmup 20 > gpurun_out/rehearse_graph.log 2>&1 || { echo "graph rehearsal failed"; tail -40 gpurun_out/rehearse_graph.log; exit 1; }
tail -2 gpurun_out/rehearse_graph.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 \
  bench.py --gpus 2 --backend gloo --mode eager --steps 100 --warmup 10 > gpurun_out/rehearse_eager.log 2>&1 || { echo "eager rehearsal failed"; tail -40 gpurun_out/rehearse_eager.log; exit 1; }
tail -1 gpurun_out/rehearse_eager.log
timeout -k 10 300 python benchmarks/job_latency.py --replicas 1 --backend rccl --gpus 0 --json-out gpurun_out/job_latency_gpu.json > gpurun_out/job_latency.log 2>&1 || { echo "latency failed"; tail -30 gpurun_out/job_latency.log; exit 1; }
cat gpurun_out/job_latency.log | tail -2
