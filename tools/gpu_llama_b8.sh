#!/bin/bash
# Llama-3 8B per-rank batch 8 (M = 16384 tokens per GEMM) vs 4 on one MI355X, both replaying
# the in-tree TunableOp winners (tuning/gemm_mi355x.csv covers both batches).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/b8v; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
L="python -u -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048"
timeout -k 10 400 $L --batch-size 8 --steps 6 --warmup 3 > $O/b8.log 2>&1 || { echo "b8 failed"; tail -20 $O/b8.log; exit 1; }
echo "b8 $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*\|"max_mem_gb": [0-9.]*\|"gemm_tuning": "[a-z]*"' $O/b8.log | tr '\n' ' ')"
timeout -k 10 400 $L --batch-size 4 --steps 8 --warmup 3 > $O/b4.log 2>&1 || { echo "b4 failed"; tail -20 $O/b4.log; exit 1; }
echo "b4 $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*\|"max_mem_gb": [0-9.]*\|"gemm_tuning": "[a-z]*"' $O/b4.log | tr '\n' ' ')"
