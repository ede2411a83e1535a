#!/bin/bash
# Round 4 session 25: conv12_fwd conv1 MFMA tiles balanced against the VALU windows (in-tree)
# vs the round-robin layout (exp/c1bal0.so): kernel tests, timelines, bench (ab_libs.sh), and
# the per-wave conv1 stamps of the balanced layout.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s25; mkdir -p $O
export PYTHONUNBUFFERED=1
PTO_HIP_LIB=$GRAFT_REPO_ROOT/pytorch_operator_amd/_lib/diag/mnist_stampw.so timeout -k 10 200 python tools/step_timeline.py --conv1-waves --reps 3 > $O/stampw.txt 2>&1 || { tail -20 $O/stampw.txt; exit 1; }
grep "conv1 per-wave" $O/stampw.txt
bash tools/gpu/ab_libs.sh $O/ab 2
