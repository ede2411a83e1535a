#!/bin/bash
# Same-box A/B of the world-2 bucketed all-reduce step (FlatGradAllReduce: G1 / fc bucket /
# G2 / conv bucket / G3) with the three pieces replayed as hipGraphs (--launch graph) vs
# their kernel lists launched straight onto the stream (--launch stream).  Both ranks share
# the box's GPU, so the process group is gloo; REPS interleaved repetitions.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
REPS=${REPS:-3}
port=29611
for rep in $(seq $REPS); do
for launch in graph stream; do
  port=$((port + 1))
  v="$(timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
       --master-port $port bench.py --gpus 2 --backend gloo --allreduce rccl --launch $launch --steps 200 \
       --warmup 20 --job-latency 0 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1
  echo "launch=$launch | world 2 gloo rccl-path K200: $v ms/step" | tee -a gpurun_out/split_ab.txt
done
done
