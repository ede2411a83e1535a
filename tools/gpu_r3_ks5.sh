#!/bin/bash
# Round 3: MNIST variant libraries -- fc1 split-K 5 (640 workgroups of 2 waves) and the head's
# DPP/permlane logit all-reduce -- numerics of every variant, then the same-box bench A/B
# (tools/gpu_ab_libs2.sh: in-tree vs exp/*.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in pytorch_operator_amd/_lib/exp/*.so; do
PTO_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "not fc1_bwd_head and not fused_schedule" --timeout 120 --timeout-method thread > gpurun_out/var_test.log 2>&1 || { echo "tests failed with $lib"; tail -30 gpurun_out/var_test.log; exit 1; }
echo "$lib: $(tail -1 gpurun_out/var_test.log)"
done
REPS=3 timeout -k 10 1000 bash tools/gpu_ab_libs2.sh
