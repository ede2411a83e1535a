#!/bin/bash
# Round 3: Llama-3 8B step (B=4, seq 2048, world 1, MasterAdamW path) with the round-2 attention
# kernels (PTO_ATTN_FWD=4: 4-wave forward and dQ pass) vs the round-3 defaults, same box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3l; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
L="python -u -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4 --steps 8 --warmup 3 --zero 0"
# r2: the round-2 attention kernels (4-wave forward + dQ, plain dK/dV, AGPR-form build)
for rep in 1 2; do for arm in r2 r3; do
if [ $arm = r2 ]; then E="PTO_HIP_LIB=pytorch_operator_amd/_lib/exp/attn_agpr.so PTO_ATTN_FWD=4 PTO_ATTN_DKDV=1"; else E=""; fi
env $E timeout -k 10 300 $L > $O/l_$arm.log 2>&1 || { echo "llama $arm failed"; tail -20 $O/l_$arm.log; exit 1; }
echo "VARIANT llama attn=$arm rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*\|"max_mem_gb": [0-9.]*' $O/l_$arm.log | tr '\n' ' ')"
done; done
