#!/bin/bash
# ResNet-50 bf16 variants on one MI355X (B=256, 224x224).  MIOpen's find results go to
# gpurun_out/miopen (MIOPEN_USER_DB_PATH) so a searched database can be inspected / kept.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/resnet gpurun_out/miopen
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/gpurun_out/miopen MIOPEN_CUSTOM_CACHE_DIR=$GRAFT_REPO_ROOT/gpurun_out/miopen
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
run() { s=$(date +%s); timeout -k 10 420 python -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 20 --warmup 8 "$@" > gpurun_out/resnet/out.log 2>gpurun_out/resnet/err.log; rc=$?; grep '"metric"' gpurun_out/resnet/out.log; echo "wall $(( $(date +%s) - s )) s rc=$rc"; return $rc; }
for v in "$@"; do
  echo "== $v"; run $v || { tail -20 gpurun_out/resnet/err.log; exit 1; }
done
