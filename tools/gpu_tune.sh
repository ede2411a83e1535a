#!/bin/bash
# Llama-3 8B (B=4, S=2048) on one MI355X: fused cross-entropy check, then hipBLASLt/rocBLAS
# GEMM selection through TunableOp: untuned -> tune (writes gpurun_out/tuning/*.csv) -> use.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tune
O=gpurun_out/tune
( while sleep 30; do echo "hb $(date +%T)" >> $O/heartbeat.txt; echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_llm_gpu.py tests/test_attention_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L="python -u -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4"
timeout -k 10 400 $L --steps 6 --warmup 3 --gemm-tuning off > $O/llama_off.log 2>&1 || { echo "llama off failed"; tail -20 $O/llama_off.log; exit 1; }
grep '"metric"' $O/llama_off.log
export PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0
cp pytorch_operator_amd/tuning/gemm_mi355x.csv $O/gemm_mi355x.csv
timeout -k 10 900 $L --steps 3 --warmup 2 --gemm-tuning tune --gemm-tuning-file $O/gemm_mi355x.csv > $O/llama_tune.log 2>&1 || { echo "llama tune failed"; tail -20 $O/llama_tune.log; exit 1; }
grep '"metric"' $O/llama_tune.log
timeout -k 10 400 $L --steps 6 --warmup 3 --gemm-tuning use --gemm-tuning-file $O/gemm_mi355x.csv > $O/llama_use.log 2>&1 || { echo "llama use failed"; tail -20 $O/llama_use.log; exit 1; }
grep '"metric"' $O/llama_use.log
