#!/bin/bash
# Round 5: end-of-round model numbers on one MI355X (Llama-3 8B batch 4 and 8, ResNet-50 batch 256).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
RUN_TIMEOUT=500 bash tools/gpu/models.sh gpurun_out/r5_models \
  "--model llama3-8b --seq-len 2048 --batch-size 4 --steps 8 --warmup 3 --zero 0" \
  "--model llama3-8b --seq-len 2048 --batch-size 8 --steps 6 --warmup 3 --zero 0" \
  "--model resnet50 --batch-size 256 --steps 20 --warmup 8"
