#!/bin/bash
# Round 4 session 24: conv12_fwd's conv1 phase per wave (diagnostic stamps build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s24; mkdir -p $O
export PYTHONUNBUFFERED=1
PTO_HIP_LIB=$GRAFT_REPO_ROOT/pytorch_operator_amd/_lib/exp/stampw.so timeout -k 10 200 python tools/step_timeline.py --conv1-waves --reps 3 > $O/timeline.txt 2>&1 || { tail -20 $O/timeline.txt; exit 1; }
grep -E "conv1 per-wave|conv12_fwd" $O/timeline.txt | head -12
