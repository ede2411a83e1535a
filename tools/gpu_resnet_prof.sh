#!/bin/bash
# ResNet-50: numerics tests (unless SKIP_TESTS), one run that fills MIOpen's find database,
# then a rocprofv3 kernel-stats profile of the steady bf16 B=256 step (10 timed + 5 warm-up).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/rprof /tmp/miopen
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
export MIOPEN_USER_DB_PATH=/tmp/miopen MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_resnet_gpu.py -m gpu > gpurun_out/resnet_test.log 2>&1; rc=$?
  tail -8 gpurun_out/resnet_test.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 500 python3 -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 5 --warmup 3 "$@" > gpurun_out/rprof/find.log 2>&1 || { tail -20 gpurun_out/rprof/find.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/rprof -o run --output-format csv -- python3 -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 10 --warmup 5 "$@" > gpurun_out/rprof/out.log 2>&1 || { tail -20 gpurun_out/rprof/out.log; exit 1; }
grep '"metric"' gpurun_out/rprof/out.log
f=$(find /tmp/rprof -name "*kernel_trace.csv" | head -1)
python3 tools/kstats_summary.py --trace "$f" FusedSgd 8 15 | tee gpurun_out/rprof/summary_${TAG:-run}.md; rm -rf /tmp/rprof
