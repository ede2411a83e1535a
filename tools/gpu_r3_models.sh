#!/bin/bash
# Round-3 large-model A/Bs on one MI355X: ZeRO-1 gradient-as-bucket-view (Llama-3 8B B=4,
# world 1) vs the copy path vs MasterAdamW; ResNet-50 B=256 bf16 with the residual gradient
# summed in bn3's backward (GradLink) vs autograd's add pass.  VARIANT lines to stdout.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3m; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_llm_gpu.py tests/test_batchnorm_gpu.py -x -q --timeout 200 --timeout-method thread -k "zero or residual or resnet_blocks" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
R="python -u -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 20 --warmup 8"
for rep in 1 2; do for v in 1 0; do
timeout -k 10 300 $R --bn-link $v > $O/rn_link$v.log 2>&1 || { echo "resnet link=$v failed"; tail -20 $O/rn_link$v.log; exit 1; }
echo "VARIANT resnet bn_link=$v rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/rn_link$v.log | tr '\n' ' ')"
done; done
[ -n "$SKIP_LLAMA" ] && exit 0
L="python -u -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4 --steps 8 --warmup 3"
for v in "--zero 1" "--zero 1 --zero-grad-view 0" "--zero 0"; do
n=$(echo $v | tr -d ' -')
timeout -k 10 300 $L $v > $O/l_$n.log 2>&1 || { echo "llama $v failed"; tail -20 $O/l_$n.log; exit 1; }
echo "VARIANT llama $v $(grep -o '"ms_per_step": [0-9.]*\|"max_mem_gb": [0-9.]*\|"optimizer_state_gb_per_rank": [0-9.]*\|"zero_grad_sinks": [0-9]*' $O/l_$n.log | tr '\n' ' ')"
done
