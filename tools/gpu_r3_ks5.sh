#!/bin/bash
# Round 3: fc1 split-K 5 (640 workgroups of 2 waves) vs 2 -- numerics of the variant library,
# then the same-box bench A/B (tools/gpu_ab_libs2.sh: in-tree vs exp/*.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PTO_HIP_LIB=pytorch_operator_amd/_lib/exp/ks5.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ks5_test.log 2>&1 || { echo "ks5 tests failed"; tail -30 gpurun_out/ks5_test.log; exit 1; }
tail -1 gpurun_out/ks5_test.log
REPS=3 timeout -k 10 900 bash tools/gpu_ab_libs2.sh
