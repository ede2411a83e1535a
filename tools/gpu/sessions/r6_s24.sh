#!/bin/bash
# round 6: conv_bwd4 group A (2a, the critical path) at raised wave priority over group B's 2b
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s24}; mkdir -p $O
export PYTHONUNBUFFERED=1
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
TL_ARGS="--by-mod conv_bwd4:4" bash tools/gpu/ab_libs.sh $O/ab 2 || exit 1
