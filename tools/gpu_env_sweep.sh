#!/bin/bash
# HIP runtime settings vs the graph-replayed MNIST step (bench K=2000 and K=20)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/env
run() {
  local tag=$1; shift
  local a b
  a=$(env "$@" timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --job-latency 0 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || { echo "$tag failed"; return 1; }
  b=$(env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --job-latency 0 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || { echo "$tag failed"; return 1; }
  echo "$tag | K2000 $a | K20 $b"
}
run baseline X=1 &&
run devkernarg1 HIP_FORCE_DEV_KERNARG=1 &&
run devkernarg0 HIP_FORCE_DEV_KERNARG=0 &&
run pktcapture1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 &&
run pktcapture0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 &&
run hdpwa0 DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0 &&
run directdispatch0 AMD_DIRECT_DISPATCH=0 &&
run baseline2 X=1
