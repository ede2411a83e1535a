#!/bin/bash
# Llama-3 8B B=4 per-kernel profile (3 training steps: 1 first + 1 warm-up + 1 timed) and a
# ResNet-50 B=256 throughput check, one MI355X.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/llmprof2; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- \
  python3 -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4 --steps 1 --warmup 2 \
  > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
grep '"metric"' $O/prof.log
for r in fused plain fused plain; do
timeout -k 10 400 python3 -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4 --steps 6 --warmup 3 --residual-norm $r \
  > $O/llama_$r.log 2>&1 || { echo "llama $r failed"; tail -20 $O/llama_$r.log; exit 1; }
echo "$r $(grep -o '"ms_per_step": [0-9.]*' $O/llama_$r.log)"
done
timeout -k 10 420 python3 -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 20 --warmup 8 \
  > $O/resnet50.log 2>&1 || { echo "resnet failed"; tail -20 $O/resnet50.log; exit 1; }
grep '"metric"' $O/resnet50.log
