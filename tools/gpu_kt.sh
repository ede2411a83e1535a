#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu > gpurun_out/pytest_kt.log 2>&1
grep -E "PASS|FAIL|passed|failed|AssertionError" gpurun_out/pytest_kt.log | head -20
