#!/bin/bash
# Round-3 ResNet-50 B=256 bf16 A/B: residual+ReLU BN backward masks from a 1-bit forward image
# (--bn-mask bits) vs re-read from the BN output (output); BN GPU tests first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3t; mkdir -p $O /tmp/miopen
export MIOPEN_USER_DB_PATH=/tmp/miopen MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_batchnorm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
R="python -u -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 20 --warmup 8"
for rep in 1 2; do for v in bits output; do
timeout -k 10 300 $R --bn-mask $v > $O/rn.log 2>&1 || { echo "resnet $v failed"; tail -20 $O/rn.log; exit 1; }
echo "VARIANT resnet bn_mask=$v rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/rn.log | tr '\n' ' ')"
done; done
