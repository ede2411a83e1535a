#!/bin/bash
# Host completion wait: ROC_ACTIVE_WAIT_TIMEOUT (spin before the interrupt wait) vs default,
# driver-config bench (K=20, W=5) alternated, plus K=2000.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/wait; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
run() {
  local tag=$1 k=$2 w=$3; shift 3
  env "$@" timeout -k 10 120 python bench.py --steps $k --warmup $w --job-latency 0 > $O/${tag}_$k.log 2>&1 || { echo "$tag failed"; tail -5 $O/${tag}_$k.log; return 1; }
  echo "$tag K=$k $(grep -o '"ms_per_step": [0-9.]*' $O/${tag}_$k.log)"
}
for r in 1 2 3; do
  run default 20 5 X=1 || exit 1
  run spin 20 5 ROC_ACTIVE_WAIT_TIMEOUT=100000 || exit 1
done
run default 2000 50 X=1 && run spin 2000 50 ROC_ACTIVE_WAIT_TIMEOUT=100000
