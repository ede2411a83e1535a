#!/bin/bash
# Model throughput runs on one MI355X through the DDP trainer harness, one run per argument
# string, e.g.
#   bash tools/gpu/models.sh OUT_DIR "--model resnet50 --batch-size 256 --steps 20 --warmup 8" \
#                                    "--model llama3-8b --seq-len 2048 --batch-size 1 --steps 5 --warmup 2"
# MIOpen's find database goes to OUT_DIR/miopen.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$1; shift; mkdir -p $O/miopen
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/$O/miopen MIOPEN_CUSTOM_CACHE_DIR=$GRAFT_REPO_ROOT/$O/miopen
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
i=0
for v in "$@"; do
  i=$((i+1)); s=$(date +%s)
  timeout -k 10 ${RUN_TIMEOUT:-600} python -m pytorch_operator_amd.harness.ddp_train $v > $O/run$i.log 2>$O/run$i.err
  rc=$?; echo "== $v"; grep '"metric"' $O/run$i.log; echo "wall $(( $(date +%s) - s )) s rc=$rc"
  [ $rc -ne 0 ] && { tail -20 $O/run$i.err; exit $rc; }
done
exit 0
