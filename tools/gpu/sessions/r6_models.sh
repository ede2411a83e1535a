#!/bin/bash
# round 6, end of session: the large-model workers on this tree (same arguments as round 5)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
RUN_TIMEOUT=500 bash tools/gpu/models.sh gpurun_out/r6_models \
  "--model llama3-8b --seq-len 2048 --batch-size 4 --steps 8 --warmup 3 --zero 0" \
  "--model llama3-8b --seq-len 2048 --batch-size 8 --steps 6 --warmup 3 --zero 0" \
  "--model resnet50 --batch-size 256 --steps 20 --warmup 8"
