#!/bin/bash
# Round 4 session 35: the 8-wave forward with LDS-DMA K/V staging (forward variant 10) vs the
# register-staged one (8): attention tests, interleaved attn_bench, kernel times.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s35; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_attn.log 2>&1
rc=$?; tail -2 $O/pytest_attn.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/pytest_attn.log | head; exit $rc; }
for rep in 1 2 3; do for v in 8 10; do
  PTO_ATTN_FWD=$v PROF_TIMEOUT=120 TOP=4 bash tools/gpu/profile.sh $O/prof_${v}_$rep 0 python3 tools/attn_bench.py --impl hip --reps 10 > $O/prof_${v}_$rep.log 2>&1 || { tail -20 $O/prof_${v}_$rep.log; exit 1; }
  echo "fwd $v rep $rep: $(grep -E 'attn_fwd8' $O/prof_${v}_$rep/kernel_stats.md)"
done; done
