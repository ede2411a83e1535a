#!/bin/bash
# Round 3: dK/dV lean pass at one (variant 4) vs two (variant 5, V from LDS) waves per SIMD;
# numerics tests of every dK/dV variant first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3g; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread -k dkdv > $O/attn_test.log 2>&1 || { echo "attn tests failed"; grep -E "FAIL|Error|assert" $O/attn_test.log | head -20; tail -30 $O/attn_test.log; exit 1; }
tail -1 $O/attn_test.log
for rep in 1 2; do for v in 4 5; do
PTO_ATTN_DKDV=$v timeout -k 10 200 python tools/attn_bench.py --impl hip > $O/a.log 2>&1 || { echo "attn bench dkdv $v failed"; tail -20 $O/a.log; exit 1; }
echo "VARIANT dkdv=$v $(tail -1 $O/a.log)"
done; done
