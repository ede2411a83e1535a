#!/bin/bash
# Attention kernels: timing + rocprofv3 kernel trace of the HIP path at the 8B shape.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/attn_prof
if [ "${1:-}" = test ]; then
  timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_test.log 2>&1 || { tail -30 gpurun_out/attn_test.log; exit 1; }
  tail -2 gpurun_out/attn_test.log
fi
timeout -k 10 200 python tools/attn_bench.py --impl hip --json-out gpurun_out/attn_bench.json > gpurun_out/attn_bench.log 2>&1 || { tail -20 gpurun_out/attn_bench.log; exit 1; }
tail -1 gpurun_out/attn_bench.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/attn_prof -o run -- python3 tools/attn_bench.py --impl hip --reps 5 > gpurun_out/attn_prof/log 2>&1 || { tail -20 gpurun_out/attn_prof/log; exit 1; }
find gpurun_out/attn_prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -12
