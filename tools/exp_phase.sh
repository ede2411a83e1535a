#!/bin/bash
# Kernel A/B: phase profile + bench for the in-tree library and every variant in
# pytorch_operator_amd/_lib/exp/*.so (built with -D experiment macros).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for lib in "" $(ls pytorch_operator_amd/_lib/exp/*.so 2>/dev/null); do
  echo "=== ${lib:-baseline}"
  PTO_HIP_LIB=$lib timeout -k 10 120 python tools/phase_profile.py 2>&1 | grep -v amdgpu.ids || exit 1
  for rep in 1 2; do PTO_HIP_LIB=$lib timeout -k 10 120 python bench.py --steps 4000 --warmup 100 2>&1 | grep -o "\"ms_per_step\": [0-9.]*" || exit 1; done
done
