#!/bin/bash
# GPU: Llama-3 8B per-kernel profile (B=1) + batch sweep (B=2,4) on one MI355X
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/llmprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/llmprof/p -o run --output-format csv -- \
  python3 -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 1 --steps 3 --warmup 2 \
  > gpurun_out/llmprof/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/llmprof/prof.log; exit 1; }
tail -1 gpurun_out/llmprof/prof.log
for b in 2 4; do
  timeout -k 10 600 python3 -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size $b \
    --steps 4 --warmup 2 > gpurun_out/llmprof/b$b.log 2>&1 || { echo "B=$b failed"; tail -20 gpurun_out/llmprof/b$b.log; exit 1; }
  tail -1 gpurun_out/llmprof/b$b.log
done
