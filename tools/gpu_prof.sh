#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run -- python3 bench.py --steps 500 --warmup 20 --mode eager > $R/gpurun_out/prof/bench.log 2>&1
rc=$?
tail -5 $R/gpurun_out/prof/bench.log
find $R/gpurun_out/prof -name "*stats*" | head
exit $rc
