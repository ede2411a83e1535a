#!/bin/bash
# Round 4 session 19: pipelined dK/dV pass variants (transposed-read lead 4 / 6 / 8 gaps, no
# s_nop pad before the first dV / dK MFMA of a k-step): numerics on each, interleaved attn_bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s19; mkdir -p $O
export PYTHONUNBUFFERED=1
D=$GRAFT_REPO_ROOT/pytorch_operator_amd/_lib/diag
for v in lead6 lead8 nopad; do
  PTO_HIP_LIB=$D/$v.so timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread -k "dkdv_variants and 8 or bit_identical" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do for v in base lead6 lead8 nopad; do
  L=""; [ $v != base ] && L=$D/$v.so
  PTO_HIP_LIB=$L timeout -k 10 200 python tools/attn_bench.py --impl hip --json-out $O/attn_${v}_$rep.json > $O/attn_${v}_$rep.log 2>&1 || { tail -20 $O/attn_${v}_$rep.log; exit 1; }
  echo "$v rep $rep: $(tail -1 $O/attn_${v}_$rep.log | grep -o '"bwd_us": [0-9.]*')"
done; done
