#!/bin/bash
# GPU: RMSNorm/LLM tests + ResNet-50 and Llama-3 throughput on one MI355X
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_llm_gpu.py -x -q > gpurun_out/llm_pytest.log 2>&1 || { echo "llm tests failed"; tail -40 gpurun_out/llm_pytest.log; exit 1; }
tail -2 gpurun_out/llm_pytest.log
timeout -k 10 300 python -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 20 --warmup 5 > gpurun_out/resnet50.log 2>&1 || { echo "resnet failed"; tail -20 gpurun_out/resnet50.log; exit 1; }
tail -1 gpurun_out/resnet50.log
timeout -k 10 600 python -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 1 --steps 5 --warmup 2 > gpurun_out/llama8b.log 2>&1 || { echo "llama8b failed"; tail -20 gpurun_out/llama8b.log; exit 1; }
tail -1 gpurun_out/llama8b.log
