#!/bin/bash
# round 6: where the fixed cost of the K=20 timed region goes (t(K) = a + b K), and a HIP
# runtime + kernel trace of bench.py --steps 20
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s10}; mkdir -p $O
export PYTHONUNBUFFERED=1
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python tools/dbg/k_sweep.py > $O/k_sweep.json 2> $O/k_sweep.err || { tail -20 $O/k_sweep.err; exit 1; }
cat $O/k_sweep.json
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 5 --job-latency 0 > $O/trace_bench.log 2>&1 || { tail -20 $O/trace_bench.log; exit 1; }
grep '^{"metric' $O/trace_bench.log | cut -c1-200
find $O/trace -name "*.csv" | head
