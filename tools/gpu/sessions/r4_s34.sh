#!/bin/bash
# Round 4 session 34: PMC counters of the final attention kernels (both pipelined backward
# passes and the forward) on the 8B shape.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/pmc.sh gpurun_out/r4s34/pmc python3 tools/attn_bench.py --impl hip --reps 5 > gpurun_out/r4s34_pmc.log 2>&1 || { tail -20 gpurun_out/r4s34_pmc.log; exit 1; }
grep -A 18 "attn_" gpurun_out/r4s34/pmc/summary.txt | head -70
