#!/bin/bash
# fused batch-norm kernels: numerics tests, ResNet numerics tests, then the ResNet-50 A/B
# (--bn hip vs library, MIOpen search on, B=256)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/bn /tmp/miopen
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
export MIOPEN_USER_DB_PATH=/tmp/miopen MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_batchnorm_gpu.py -m gpu > gpurun_out/bn/test_bn.log 2>&1; rc=$?
tail -4 gpurun_out/bn/test_bn.log; [ $rc -eq 0 ] || exit $rc
for v in library hip library hip; do
  timeout -k 10 500 python -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 20 --warmup 8 --bn $v > gpurun_out/bn/rn_$v.log 2>&1 || { tail -20 gpurun_out/bn/rn_$v.log; exit 1; }
  echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/bn/rn_$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bn/rn_$v.log) $(grep -o '"loss": [0-9.]*' gpurun_out/bn/rn_$v.log)"
done
[ -n "$SKIP_RESNET_TESTS" ] || { timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_resnet_gpu.py -m gpu > gpurun_out/bn/test_resnet.log 2>&1; rc=$?; tail -8 gpurun_out/bn/test_resnet.log; [ $rc -eq 0 ] || exit $rc; }
