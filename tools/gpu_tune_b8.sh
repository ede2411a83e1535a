#!/bin/bash
# TunableOp search for the Llama-3 8B batch-8 GEMM shapes not yet in the table (backward
# shapes), bounded; partial results survive in the .tuning file.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/tune8; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
cp pytorch_operator_amd/tuning/gemm_mi355x.csv $O/gemm.csv
timeout -k 10 ${TUNE_S:-900} python -u -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 8 --steps 1 --warmup 1 --gemm-tuning tune --gemm-tuning-file $O/gemm.csv > $O/tune.log 2>&1
echo "tune rc=$? tuned lines: $(grep -vc Validator $O/gemm.csv.tuning 2>/dev/null)"
exit 0
