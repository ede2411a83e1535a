#!/bin/bash
# round 6: K=20 against the pre-warm duration (bench.py --prewarm-ms), interleaved x3
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s28}; mkdir -p $O
for rep in 1 2 3; do
  for pw in 0 10 40 100 250; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --job-latency 0 --prewarm-ms $pw > $O/b_${pw}_$rep.log 2>&1 || exit 1
    echo "prewarm $pw: $(grep -o '"ms_per_step": [0-9.]*' $O/b_${pw}_$rep.log)"
  done
done
