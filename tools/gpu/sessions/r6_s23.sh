#!/bin/bash
# round 6: end-of-region waits at K=20 incl. spinning on a pinned host flag (k_sweep --brackets)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s23}; mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  timeout -k 10 200 python tools/dbg/k_sweep.py --ks 20,2000 --reps 15 > $O/k_$rep.json 2>$O/k_$rep.err || { tail $O/k_$rep.err; exit 1; }
  cat $O/k_$rep.json
done
