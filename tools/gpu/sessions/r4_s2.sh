#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s2; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_kernels.log 2>&1
rc=$?; tail -3 $O/pytest_kernels.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_libs.sh $O 2
