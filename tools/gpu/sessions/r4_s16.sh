#!/bin/bash
# Round 4 session 16: in-kernel stamps of the pipelined dK/dV pass (diagnostic build), and the
# Llama-3 8B step with dK/dV variant 7 vs 8 (interleaved, same box).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s16; mkdir -p $O
export PYTHONUNBUFFERED=1
PTO_HIP_LIB=$GRAFT_REPO_ROOT/pytorch_operator_amd/_lib/diag/attn_stamps.so timeout -k 10 200 python tools/attn_pipe_stamps.py --json $O/stamps.json > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
for rep in 1 2; do for v in 7 8; do
  PTO_ATTN_DKDV=$v RUN_TIMEOUT=400 bash tools/gpu/models.sh $O/llama_${v}_$rep "--model llama3-8b --seq-len 2048 --batch-size 4 --steps 8 --warmup 3 --zero 0" || exit 1
done; done
