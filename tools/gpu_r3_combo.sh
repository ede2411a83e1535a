#!/bin/bash
# Round 3 combined call: ZeRO arrival debug, attention tests + A/B (4-wave vs 8-wave fwd/dQ),
# MNIST step A/B (variant libs + fc-sgd flags).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3c; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 120 --timeout-method thread > $O/attn_test.log 2>&1 || { echo "attn tests failed"; tail -40 $O/attn_test.log; exit 1; }
tail -1 $O/attn_test.log
for v in 8 9 8 9; do
PTO_ATTN_FWD=$v timeout -k 10 200 python tools/attn_bench.py --impl hip --json-out $O/attn_$v.json > $O/attn_$v.log 2>&1 || { echo "attn bench $v failed"; tail -20 $O/attn_$v.log; exit 1; }
echo "VARIANT fwd=$v $(tail -1 $O/attn_$v.log)"
done
[ -n "$MNIST_AB" ] && timeout -k 10 900 bash tools/gpu_r3_mnist_ab.sh
true
