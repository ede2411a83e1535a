#!/bin/bash
# Round 4 session 9: wave priority for conv_bwd4's group A on the software-pipelined split.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s9; mkdir -p $O
export PYTHONUNBUFFERED=1
bash tools/gpu/ab_libs.sh $O/ab 2 || exit 1
