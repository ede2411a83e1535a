#!/bin/bash
# Round 3: every dK/dV variant (1 plain, 2 software-pipelined, 3 8-wave, 4 lean) and both 8-wave
# forwards (8 barrier-aligned, 9 ping-pong) re-measured on the VGPR-form MFMA build (in-tree
# library), two interleaved repetitions at the Llama-3 8B shape.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3f; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
for rep in 1 2; do
  for v in 1 2 3 4; do
    PTO_ATTN_DKDV=$v timeout -k 10 200 python tools/attn_bench.py --impl hip > $O/a.log 2>&1 || { echo "attn bench dkdv $v failed"; tail -20 $O/a.log; exit 1; }
    echo "VARIANT fwd=8 dkdv=$v $(tail -1 $O/a.log)"
  done
  PTO_ATTN_FWD=9 timeout -k 10 200 python tools/attn_bench.py --impl hip > $O/a.log 2>&1 || { echo "attn bench fwd 9 failed"; tail -20 $O/a.log; exit 1; }
  echo "VARIANT fwd=9 dkdv=4 $(tail -1 $O/a.log)"
done
