#!/bin/bash
# Round 3: ZeRO-1 with lazily allocated gradient buckets -- GPU tests, then Llama-3 8B B=4 world 1:
# ZeRO (grad view) vs MasterAdamW, ms/step and peak memory.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3z; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 200 --timeout-method thread -k "zero or master" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L="python -u -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4 --steps 8 --warmup 3"
for v in "--zero 1" "--zero 0"; do
n=$(echo $v | tr -d ' -')
timeout -k 10 300 $L $v > $O/l_$n.log 2>&1 || { echo "llama $v failed"; tail -20 $O/l_$n.log; exit 1; }
echo "VARIANT llama $v $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*\|"max_mem_gb": [0-9.]*\|"zero_grad_sinks": [0-9]*' $O/l_$n.log | tr '\n' ' ')"
done
