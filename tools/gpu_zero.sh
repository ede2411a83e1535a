#!/bin/bash
# ZeRO-1 optimizer on one MI355X: numerics test vs MasterAdamW, then Llama-3 8B B=4 with the
# sharded optimizer path (world 1: same update work, + fp32 gradient buckets) vs the default.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/zero; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 200 --timeout-method thread -k "zero or overlap" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L="python -u -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4 --steps 8 --warmup 3"
for m in 1 0; do
timeout -k 10 300 $L --zero $m > $O/l_zero$m.log 2>&1 || { echo "llama zero=$m failed"; tail -20 $O/l_zero$m.log; exit 1; }
echo "zero=$m $(grep -o '"ms_per_step": [0-9.]*\|"max_mem_gb": [0-9.]*\|"optimizer_state_gb_per_rank": [0-9.]*' $O/l_zero$m.log | tr '\n' ' ')"
done
