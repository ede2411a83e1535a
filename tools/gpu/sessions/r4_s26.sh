#!/bin/bash
# Round 4 session 26: conv1 channels 16-19 as channel pairs on v_pk_fma_f32 (in-tree) vs the
# one-channel VALU windows (exp/c1pk0.so): kernel tests, timelines, bench (ab_libs.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s26; mkdir -p $O
export PYTHONUNBUFFERED=1
bash tools/gpu/ab_libs.sh $O/ab 2
