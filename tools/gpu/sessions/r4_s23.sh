#!/bin/bash
# Round 4 session 23: placement of the dK/dV pipeline's per-tile LDS-DMA (first gap / spacing):
# 8/1 (default), 0/1, 2/3, 16/1, 0/2.  Kernel time per build (rocprofv3), two rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s23; mkdir -p $O
export PYTHONUNBUFFERED=1
D=$GRAFT_REPO_ROOT/pytorch_operator_amd/_lib/diag
for v in dma0 dma2s3 dma16 dma0s2; do
  PTO_HIP_LIB=$D/$v.so timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread -k "dkdv_variants and 8 or bit_identical" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2; do for v in base dma0 dma2s3 dma16 dma0s2; do
  L=""; [ $v != base ] && L=$D/$v.so
  PTO_HIP_LIB=$L PROF_TIMEOUT=120 TOP=3 bash tools/gpu/profile.sh $O/prof_${v}_$rep 0 python3 tools/attn_bench.py --impl hip --reps 10 > $O/prof_${v}_$rep.log 2>&1 || { tail -20 $O/prof_${v}_$rep.log; exit 1; }
  echo "$v rep $rep: $(grep dkdv_pipe $O/prof_${v}_$rep/kernel_stats.md)"
done; done
