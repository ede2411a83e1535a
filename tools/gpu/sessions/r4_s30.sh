#!/bin/bash
# Round 4 session 30: lse2 / delta staged once per four query tiles in the pipelined dK/dV pass
# (diag/stat4.so) vs per tile (in-tree): attention tests on the variant (bit identity), kernel
# times interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s30; mkdir -p $O
export PYTHONUNBUFFERED=1
D=$GRAFT_REPO_ROOT/pytorch_operator_amd/_lib/diag
PTO_HIP_LIB=$D/stat4.so timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_attn.log 2>&1
rc=$?; tail -2 $O/pytest_attn.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/pytest_attn.log | head; exit $rc; }
for rep in 1 2 3; do for v in base stat4; do
  L=""; [ $v != base ] && L=$D/$v.so
  PTO_HIP_LIB=$L PROF_TIMEOUT=120 TOP=4 bash tools/gpu/profile.sh $O/prof_${v}_$rep 0 python3 tools/attn_bench.py --impl hip --reps 10 > $O/prof_${v}_$rep.log 2>&1 || { tail -20 $O/prof_${v}_$rep.log; exit 1; }
  echo "$v rep $rep: $(grep -E 'dkdv_pipe' $O/prof_${v}_$rep/kernel_stats.md)"
done; done
