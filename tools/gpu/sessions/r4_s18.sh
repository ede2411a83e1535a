#!/bin/bash
# Round 4 session 18: the pipelined dK/dV pass with its VALU chains skewed across gaps:
# numerics + bit identity, attn_bench vs variant 7 (interleaved), per-phase stamps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s18; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 200 --timeout-method thread -k "dkdv" > $O/pytest_attn.log 2>&1
rc=$?; tail -5 $O/pytest_attn.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do for v in 7 8; do
  PTO_ATTN_DKDV=$v timeout -k 10 200 python tools/attn_bench.py --impl hip --json-out $O/attn_dkdv${v}_$rep.json > $O/attn_dkdv${v}_$rep.log 2>&1 || { tail -20 $O/attn_dkdv${v}_$rep.log; exit 1; }
  echo "dkdv $v rep $rep: $(tail -1 $O/attn_dkdv${v}_$rep.log)"
done; done
PTO_HIP_LIB=$GRAFT_REPO_ROOT/pytorch_operator_amd/_lib/diag/attn_stamps.so timeout -k 10 200 python tools/attn_pipe_stamps.py --json $O/stamps.json > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep -A 8 "clock_mhz\|tile9_phase_cycles_p50" $O/stamps.log
