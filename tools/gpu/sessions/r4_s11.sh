#!/bin/bash
# Round 4 session 11: conv_bwd4 2a on all 16 waves before the group split; fc1_bwd fc2 + stats
# blocks first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s11; mkdir -p $O
export PYTHONUNBUFFERED=1
bash tools/gpu/ab_libs.sh $O/ab 2 || exit 1
