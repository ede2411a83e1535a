#!/bin/bash
# round 6: kernel stats of the DDP step forms -- forced single-rank RCCL (fused form: five launches,
# one all-reduce, the SGD launch) and two ranks over xGMI on the shared GPU (fused form: five)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s29}; mkdir -p $O
export PYTHONUNBUFFERED=1
PROF_TIMEOUT=300 bash tools/gpu/profile.sh $O/rccl_w1 0 python3 bench.py --gpus 1 --backend nccl --force-collectives 1 --allreduce rccl --steps 400 --warmup 40 --job-latency 0 || exit 1
PTO_XGMI_ANY_BACKEND=1 PROF_TIMEOUT=300 bash tools/gpu/profile.sh $O/xgmi_w2 0 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29901 bench.py --gpus 2 --backend gloo --allreduce xgmi --steps 400 --warmup 40 --job-latency 0 || exit 1
