#!/bin/bash
# kernel numerics + xGMI rehearsal tests, phase profile, quick bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_xgmi_gpu.py tests/test_xgmi_emu_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { echo "tests failed"; grep -E "Error|assert|FAILED|Fault" gpurun_out/pytest_iter.log | head -30; tail -30 gpurun_out/pytest_iter.log; exit 1; }
tail -2 gpurun_out/pytest_iter.log
bash tools/gpu_phase.sh && bash tools/gpu_bench_quick.sh
