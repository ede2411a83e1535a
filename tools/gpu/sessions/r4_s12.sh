#!/bin/bash
# Round 4 session 12: flash-attention dK/dV split into a dV pass and a dK pass (two waves per
# SIMD each) vs the lean one-wave pass: numerics, then interleaved attn_bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s12; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 200 --timeout-method thread -k "dkdv" > $O/pytest_attn.log 2>&1
rc=$?; tail -15 $O/pytest_attn.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for v in 4 6; do
  PTO_ATTN_DKDV=$v timeout -k 10 200 python tools/attn_bench.py --impl hip --json-out $O/attn_dkdv${v}_$rep.json > $O/attn_dkdv${v}_$rep.log 2>&1 || { tail -20 $O/attn_dkdv${v}_$rep.log; exit 1; }
  echo "dkdv $v rep $rep: $(tail -1 $O/attn_dkdv${v}_$rep.log)"
done; done
PTO_ATTN_DKDV=6 PROF_TIMEOUT=200 TOP=8 bash tools/gpu/profile.sh $O/prof6 0 python3 tools/attn_bench.py --impl hip --reps 10 || exit 1
