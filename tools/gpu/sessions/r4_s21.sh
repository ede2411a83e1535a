#!/bin/bash
# Round 4 session 21: the pipelined dQ pass in 8-wave form (two waves per SIMD, qf/dO^T
# operands in AGPRs): bit identity vs the 8-wave dQ pass, numerics, interleaved attn_bench dQ
# 8 vs 9, kernel profile of 9.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s21; mkdir -p $O
export PYTHONUNBUFFERED=1
PTO_ATTN_DQ=9 timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 200 --timeout-method thread -k "dq_pass or dkdv_variants" > $O/pytest_attn.log 2>&1
rc=$?; grep -E "FAIL|Error" $O/pytest_attn.log | tail -20; tail -2 $O/pytest_attn.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do for v in 8 9; do
  PTO_ATTN_DQ=$v timeout -k 10 200 python tools/attn_bench.py --impl hip --json-out $O/attn_dq${v}_$rep.json > $O/attn_dq${v}_$rep.log 2>&1 || { tail -20 $O/attn_dq${v}_$rep.log; exit 1; }
  echo "dq $v rep $rep: $(tail -1 $O/attn_dq${v}_$rep.log | grep -o '"bwd_us": [0-9.]*')"
done; done
PTO_ATTN_DQ=9 PROF_TIMEOUT=200 TOP=6 bash tools/gpu/profile.sh $O/prof9 0 python3 tools/attn_bench.py --impl hip --reps 10 || exit 1
