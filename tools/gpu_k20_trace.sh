#!/bin/bash
# Where the fixed ~40 us of a 20-step timed region goes: HIP runtime API + kernel trace of
# the driver's bench configuration (K=20, W=5), CSV for tools/k20_gaps.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/k20
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/k20/trace -o run -- python3 bench.py --steps 20 --warmup 5 --job-latency 0 > gpurun_out/k20/bench.log 2>&1 || { tail -30 gpurun_out/k20/bench.log; exit 1; }
tail -1 gpurun_out/k20/bench.log
find gpurun_out/k20/trace -name "*.csv" | head
