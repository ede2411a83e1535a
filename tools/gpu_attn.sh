#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/attn_test.log 2>&1; rc=$?
tail -30 gpurun_out/attn_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/attn_bench.py --json-out gpurun_out/attn_bench.json > gpurun_out/attn_bench.log 2>&1; rc=$?
tail -5 gpurun_out/attn_bench.log
exit $rc
