#!/bin/bash
# Llama-3 8B B=4: TN-backward projections vs autograd layouts (after tuning the new shapes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/tn; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L="python -u -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4"
cp pytorch_operator_amd/tuning/gemm_mi355x.csv $O/gemm_mi355x.csv
PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0 timeout -k 10 700 $L --steps 2 --warmup 2 --gemm-tuning tune --gemm-tuning-file $O/gemm_mi355x.csv > $O/tune.log 2>&1 || { echo "tune failed"; tail -20 $O/tune.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"gemm_tuned_shapes": [0-9]*' $O/tune.log
for r in 1 2; do for m in tn autograd; do
timeout -k 10 300 $L --steps 6 --warmup 3 --linear-bwd $m --gemm-tuning-file $O/gemm_mi355x.csv > $O/l_${m}_$r.log 2>&1 || { echo "llama $m failed"; tail -20 $O/l_${m}_$r.log; exit 1; }
echo "$m $(grep -o '"ms_per_step": [0-9.]*' $O/l_${m}_$r.log)"
done; done
