#!/bin/bash
# Round 3: dK/dV pass A/B -- variant 1 (plain) vs 4 (lean registers + LDS-DMA), each with
# attention.hip compiled with VGPR-form MFMAs (in-tree library) and without (exp/attn_agpr.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3e; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 120 --timeout-method thread > $O/attn_test.log 2>&1 || { echo "attn tests failed"; grep -E "FAIL|Error|assert" $O/attn_test.log | head -20; tail -30 $O/attn_test.log; exit 1; }
tail -1 $O/attn_test.log
for rep in 1 2; do for lib in "" pytorch_operator_amd/_lib/exp/attn_agpr.so; do for v in 1 4; do
PTO_HIP_LIB=$lib PTO_ATTN_DKDV=$v timeout -k 10 200 python tools/attn_bench.py --impl hip > $O/a.log 2>&1 || { echo "attn bench $lib $v failed"; tail -20 $O/a.log; exit 1; }
echo "VARIANT lib=${lib:-in-tree} dkdv=$v $(tail -1 $O/a.log)"
done; done; done
