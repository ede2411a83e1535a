#!/bin/bash
# rocprofv3 kernel trace of the graph-replayed bench (steady state) + seam analysis
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/profg; mkdir -p $R/gpurun_out/profg
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profg -o run -- python3 bench.py --steps 1000 --warmup 50 > $R/gpurun_out/profg/bench.log 2>&1 || { tail -5 $R/gpurun_out/profg/bench.log; exit 1; }
DB=$(find $R/gpurun_out/profg -name "*.db" | head -1)
python3 tools/rocpd_gaps.py $DB --skip 400 | tee $R/gpurun_out/profg/gaps.md
