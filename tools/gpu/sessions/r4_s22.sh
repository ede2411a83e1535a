#!/bin/bash
# Round 4 session 22: where the pipelined dK/dV pass's time goes -- diagnostic ablation builds
# (wrong results by design, in-bounds accesses): 1 no dS arithmetic, 2 row reads for the
# transposed operands, 4 no per-tile DMA, 8 no per-tile barrier, 16 no exp2, 31 all of them.
# Kernel time of attn_bwd_dkdv_pipe_kernel from rocprofv3 per build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s22; mkdir -p $O
export PYTHONUNBUFFERED=1
D=$GRAFT_REPO_ROOT/pytorch_operator_amd/_lib/diag
for v in base abl1 abl2 abl4 abl8 abl16 abl31; do
  L=""; [ $v != base ] && L=$D/$v.so
  PTO_HIP_LIB=$L PROF_TIMEOUT=120 TOP=3 bash tools/gpu/profile.sh $O/prof_$v 0 python3 tools/attn_bench.py --impl hip --reps 10 > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  echo "$v: $(grep dkdv_pipe $O/prof_$v/kernel_stats.md)"
done
