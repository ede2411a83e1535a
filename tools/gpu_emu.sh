#!/bin/bash
# xGMI protocol at world 2/4/8 emulated on the box's GPU + the 2-rank multi-process check.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_xgmi_emu_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/xgmi_emu.log 2>&1 || { echo "emu tests failed"; tail -60 gpurun_out/xgmi_emu.log; exit 1; }
grep -E "PASS|FAIL|us per" gpurun_out/xgmi_emu.log
