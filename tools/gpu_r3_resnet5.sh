#!/bin/bash
# Round-3 ResNet-50 B=256 bf16 A/B: residual BNs' reduce pass writes g (= dz) and the dx pass
# reads it (in-tree) vs the dx pass re-reading dy, dy2 and the mask (exp/bngout0.so, -DPTO_BN_GOUT=0).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3u; mkdir -p $O /tmp/miopen
export MIOPEN_USER_DB_PATH=/tmp/miopen MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_batchnorm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
R="python -u -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 20 --warmup 8"
for rep in 1 2; do for lib in "" pytorch_operator_amd/_lib/exp/bngout0.so; do
PTO_HIP_LIB=$lib timeout -k 10 300 $R > $O/rn.log 2>&1 || { echo "resnet $lib failed"; tail -20 $O/rn.log; exit 1; }
echo "VARIANT resnet lib=${lib:-in-tree} rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/rn.log | tr '\n' ' ')"
done; done
