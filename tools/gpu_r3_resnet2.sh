#!/bin/bash
# Round-3 ResNet-50 B=256 bf16 A/B: stage-entry downsample gradient summed in the previous bn3
# (--bn-link 2 vs 1) and the head's one-pass channels-last average-pool backward (--gap fused vs
# library).  GPU numerics tests of the BN links and the ResNet first.  VARIANT lines to stdout.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3r; mkdir -p $O /tmp/miopen
export MIOPEN_USER_DB_PATH=/tmp/miopen MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 500 python -u -m pytest tests/test_batchnorm_gpu.py tests/test_resnet_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
R="python -u -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 20 --warmup 8"
for rep in 1 2; do for v in "2 fused" "1 fused" "2 library" "1 library"; do
set -- $v
timeout -k 10 300 $R --bn-link $1 --gap $2 > $O/rn.log 2>&1 || { echo "resnet $v failed"; tail -20 $O/rn.log; exit 1; }
echo "VARIANT resnet bn_link=$1 gap=$2 rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/rn.log | tr '\n' ' ')"
done; done
