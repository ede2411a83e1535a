#!/bin/bash
# round 6: price of a two-stream step structure (tools/dbg/twostream_probe.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s18}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/dbg/twostream_probe.py --steps 2000 --reps 5 > $O/probe.json 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.json
