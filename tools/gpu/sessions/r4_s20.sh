#!/bin/bash
# Round 4 session 20: the software-pipelined dQ pass (dQ variant 9): attention GPU tests (all),
# interleaved attn_bench dQ 8 vs 9, kernel profile.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s20; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest_attn.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error" $O/pytest_attn.log | tail -60; tail -3 $O/pytest_attn.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do for v in 8 9; do
  PTO_ATTN_DQ=$v timeout -k 10 200 python tools/attn_bench.py --impl hip --json-out $O/attn_dq${v}_$rep.json > $O/attn_dq${v}_$rep.log 2>&1 || { tail -20 $O/attn_dq${v}_$rep.log; exit 1; }
  echo "dq $v rep $rep: $(tail -1 $O/attn_dq${v}_$rep.log)"
done; done
PROF_TIMEOUT=200 TOP=8 bash tools/gpu/profile.sh $O/prof 0 python3 tools/attn_bench.py --impl hip --reps 10 || exit 1
