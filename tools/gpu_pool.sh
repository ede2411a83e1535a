#!/bin/bash
# Stem max-pool kernels: numerics, then ResNet-50 B=256 --pool hip vs library (alternated);
# plus the large-model checkpoint/ZeRO GPU tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pool; mkdir -p $O /tmp/miopen
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
export MIOPEN_USER_DB_PATH=/tmp/miopen MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen
timeout -k 10 300 python -u -m pytest tests/test_pool_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_pool.log 2>&1 || { echo "pool tests failed"; tail -40 $O/pytest_pool.log; exit 1; }
tail -1 $O/pytest_pool.log
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -v --timeout 300 --timeout-method thread -k "zero or checkpoint" > $O/pytest_ckpt.log 2>&1 || { echo "ckpt tests failed"; tail -40 $O/pytest_ckpt.log; exit 1; }
tail -1 $O/pytest_ckpt.log
R="python -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 20 --warmup 8"
timeout -k 10 500 $R --steps 3 --warmup 2 > $O/find.log 2>&1 || { tail -20 $O/find.log; exit 1; }
for v in library hip library hip; do
  timeout -k 10 300 $R --pool $v > $O/rn_$v.log 2>&1 || { echo "resnet $v failed"; tail -20 $O/rn_$v.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/rn_$v.log) $(grep -o '"value": [0-9.]*' $O/rn_$v.log)"
done
