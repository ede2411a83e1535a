#!/bin/bash
# kernel numerics tests, then the lib A/B (tools/gpu_ab_libs.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu > gpurun_out/kt3.log 2>&1; rc=$?
tail -3 gpurun_out/kt3.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh
