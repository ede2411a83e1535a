#!/bin/bash
# Large-model worker features on one MI355X: ZeRO-1 numerics, checkpoint/resume (HIP AdamW path).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ckpt; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -v --timeout 300 --timeout-method thread -k "zero or checkpoint or overlap" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
