#!/bin/bash
# round 6: the fixed cost of the timed region under host-wait variants (k_sweep), interleaved twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s11}; mkdir -p $O
export PYTHONUNBUFFERED=1
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
for rep in 1 2; do
  timeout -k 10 200 python tools/dbg/k_sweep.py --ks 1,5,20,200,2000 > $O/base_$rep.json 2>$O/base_$rep.err || { tail $O/base_$rep.err; exit 1; }
  echo "base    $(cat $O/base_$rep.json)"
  timeout -k 10 200 python tools/dbg/k_sweep.py --ks 1,5,20,200,2000 --spin > $O/spin_$rep.json 2>$O/spin_$rep.err || { tail $O/spin_$rep.err; exit 1; }
  echo "spin    $(cat $O/spin_$rep.json)"; tail -1 $O/spin_$rep.err
  ROC_ACTIVE_WAIT_TIMEOUT=1000 timeout -k 10 200 python tools/dbg/k_sweep.py --ks 1,5,20,200,2000 > $O/awt_$rep.json 2>$O/awt_$rep.err || { tail $O/awt_$rep.err; exit 1; }
  echo "awt1000 $(cat $O/awt_$rep.json)"
  ROC_CPU_WAIT_FOR_SIGNAL=0 timeout -k 10 200 python tools/dbg/k_sweep.py --ks 1,5,20,200,2000 > $O/cws_$rep.json 2>$O/cws_$rep.err || { tail $O/cws_$rep.err; exit 1; }
  echo "cws0    $(cat $O/cws_$rep.json)"
done
