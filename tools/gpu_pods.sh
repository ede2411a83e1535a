#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
python -c "from pytorch_operator_amd.cluster.kubelet import namespaces_available as n; print('namespaces:', n())"
timeout -k 10 600 python -u -m pytest tests/test_e2e_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_pods.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|Error|assert" gpurun_out/pytest_pods.log | head -20
exit $rc
