#!/bin/bash
# Llama-3 8B B=4: AdamW overlapped with the next forward vs serial, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ovl; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 200 --timeout-method thread -k "overlap or linear_tn or transpose" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L="python -u -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4"
for r in 1 2; do for m in on off; do
timeout -k 10 300 $L --steps 8 --warmup 3 --opt-overlap $m > $O/l_${m}_$r.log 2>&1 || { echo "llama $m failed"; tail -20 $O/l_${m}_$r.log; exit 1; }
echo "$m $(grep -o '"ms_per_step": [0-9.]*' $O/l_${m}_$r.log)"
done; done
