#!/bin/bash
# round 6: the K=20 region's tail (rare 250-300 us stalls): distribution over 300 regions,
# default runtime vs a larger device kernel-argument pool, interleaved twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s25}; mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  timeout -k 10 200 python tools/dbg/k20_tail.py > $O/base_$rep.json 2>$O/base_$rep.err || { tail $O/base_$rep.err; exit 1; }
  echo "base  $(cat $O/base_$rep.json)"
  HSA_KERNARG_POOL_SIZE=67108864 timeout -k 10 200 python tools/dbg/k20_tail.py > $O/pool_$rep.json 2>$O/pool_$rep.err || { tail $O/pool_$rep.err; exit 1; }
  echo "pool  $(cat $O/pool_$rep.json)"
done
