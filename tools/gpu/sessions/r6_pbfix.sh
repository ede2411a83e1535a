#!/bin/bash
# round 6: xGMI / bench GPU tests after the pre-exchange barrier's exit-before-deadline fix
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6_pbfix2; mkdir -p $O
( while sleep 30; do date +%T >> $O/hb; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 700 python -u -m pytest -m gpu tests/test_xgmi_gpu.py tests/test_xgmi_emu_gpu.py tests/test_bench_gpu.py \
  -v --durations=8 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -14 $O/pytest.log
exit $rc
