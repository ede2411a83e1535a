#!/bin/bash
# Batch-norm kernel bandwidth per ResNet-50 shape; then Llama-3 8B with the ZeRO-1 optimizer (world 1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/bnb; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u tools/bn_bench.py --json $O/bn_bench.json > $O/bn_bench.log 2>&1 || { echo "bn bench failed"; tail -20 $O/bn_bench.log; exit 1; }
tail -1 $O/bn_bench.log
[ -n "$SKIP_ZERO" ] && exit 0
timeout -k 10 300 python -u -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4 --steps 8 --warmup 3 --zero 1 > $O/l_zero1.log 2>&1 || { echo "llama zero failed"; tail -20 $O/l_zero1.log; exit 1; }
echo "zero=1 $(grep -o '"ms_per_step": [0-9.]*\|"max_mem_gb": [0-9.]*' $O/l_zero1.log | tr '\n' ' ')"
