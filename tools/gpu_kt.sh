#!/bin/bash
# kernel numerics tests only (fast iteration)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_kt.log 2>&1 || { echo "kernel tests failed"; grep -E "Error|assert|FAILED|Fault" gpurun_out/pytest_kt.log | head -30; tail -30 gpurun_out/pytest_kt.log; exit 1; }
tail -3 gpurun_out/pytest_kt.log
