#!/bin/bash
# Driver-contract bench (K=20, W=5) a few times + one long run; no job-latency phase unless asked.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/bq
JL=${JL:-0}
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --job-latency $JL > gpurun_out/bq/b20_$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bq/b20_$i.log; exit 1; }
  tail -1 gpurun_out/bq/b20_$i.log | cut -c1-150
done
timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --job-latency 0 > gpurun_out/bq/b2000.log 2>&1 || { echo "bench 2000 failed"; tail -20 gpurun_out/bq/b2000.log; exit 1; }
tail -1 gpurun_out/bq/b2000.log | cut -c1-150
