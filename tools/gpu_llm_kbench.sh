#!/bin/bash
# GPU: rmsnorm numerics + per-op timing of the Llama fused kernels at 8B shapes
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/llmk
timeout -k 10 300 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 120 --timeout-method thread -k "rmsnorm or rope or swiglu or fused" \
  > gpurun_out/llmk/pytest.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/llmk/pytest.log; exit 1; }
tail -2 gpurun_out/llmk/pytest.log
PYTHONPATH=$PWD timeout -k 10 200 python3 tools/llm_kernel_bench.py > gpurun_out/llmk/kbench.jsonl 2>&1 || { echo "kbench failed"; tail -30 gpurun_out/llmk/kbench.jsonl; exit 1; }
cat gpurun_out/llmk/kbench.jsonl
