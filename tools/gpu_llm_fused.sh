#!/bin/bash
# GPU: fused LLM kernel numerics (RMSNorm pairs / RoPE / SwiGLU / tiny Llama vs CPU) + Llama-3 8B
# per-kernel profile and throughput at B=4 on one MI355X
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/llmfused
timeout -k 10 300 python -u -m pytest tests/test_llm_gpu.py -x -v --timeout 120 --timeout-method thread -k "not resnet50" \
  > gpurun_out/llmfused/pytest.log 2>&1 || { echo "llm tests failed"; tail -60 gpurun_out/llmfused/pytest.log; exit 1; }
tail -3 gpurun_out/llmfused/pytest.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/llmfused/p -o run --output-format csv -- \
  python3 -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4 --steps 3 --warmup 1 \
  > gpurun_out/llmfused/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/llmfused/prof.log; exit 1; }
grep '"metric"' gpurun_out/llmfused/prof.log
timeout -k 10 400 python3 -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4 \
  --steps 6 --warmup 2 > gpurun_out/llmfused/b4.log 2>&1 || { echo "B=4 failed"; tail -20 gpurun_out/llmfused/b4.log; exit 1; }
tail -1 gpurun_out/llmfused/b4.log
