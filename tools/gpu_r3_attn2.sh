#!/bin/bash
# Round 3: attention kernels A/B -- forward 8 (plain) vs 9 (ping-pong), dK/dV 1 (4-wave) vs
# 3 (8-wave); dQ is the 8-wave LDS-DMA pass in both.  Tests first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3d; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 120 --timeout-method thread > $O/attn_test.log 2>&1 || { echo "attn tests failed"; grep -E "FAIL|Error|assert" $O/attn_test.log | head -20; tail -30 $O/attn_test.log; exit 1; }
tail -1 $O/attn_test.log
for rep in 1 2; do for v in "8 1" "9 1" "8 3" "9 3"; do
set -- $v
PTO_ATTN_FWD=$1 PTO_ATTN_DKDV=$2 timeout -k 10 200 python tools/attn_bench.py --impl hip > $O/attn_$1_$2.log 2>&1 || { echo "attn bench $v failed"; tail -20 $O/attn_$1_$2.log; exit 1; }
echo "VARIANT fwd=$1 dkdv=$2 $(tail -1 $O/attn_$1_$2.log)"
done; done
PTO_ATTN_FWD=9 PTO_ATTN_DKDV=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/attn_bench.py --impl hip --reps 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160 | head -8
