#!/bin/bash
# Round 4 session 17: per-phase stamps of one tile of the pipelined dK/dV pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s17; mkdir -p $O
export PYTHONUNBUFFERED=1
PTO_HIP_LIB=$GRAFT_REPO_ROOT/pytorch_operator_amd/_lib/diag/attn_stamps.so timeout -k 10 200 python tools/attn_pipe_stamps.py --json $O/stamps.json > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
