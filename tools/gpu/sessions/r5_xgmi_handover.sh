#!/bin/bash
# Round 5: root cause of the r4 hand-over timeouts at 2 x 256 exchange workgroups on one shared
# GPU.  Runs the rehearsal with the hand-over stage forced to the 256 geometry and the
# exchange's per-workgroup stamps on, RUNS times, and reads every timed-out launch's stamps with
# tools/xgmi_stamps.py (starvation vs a flag raised but not seen).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r5_handover}; mkdir -p $O
export PYTHONUNBUFFERED=1
port=29710
for i in $(seq 1 ${RUNS:-4}); do
  port=$((port + 1))
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port tools/xgmi_check.py --backend gloo --nblk 256 --handover-nblk ${HNB:-256} --stamps \
    --fuse-conv12 ${FUSE:--1} --out $O/run$i > $O/run$i.log 2>&1
  rc=$?
  echo "== run $i rc=$rc"; grep -ho '"error_after": {[^}]*}' $O/run$i.log | head -2
  case $rc in 0|1) ;; *) tail -20 $O/run$i.log; exit $rc;; esac
  for t in main handover; do
    [ -d $O/run$i/stamps_$t ] || continue
    python tools/xgmi_stamps.py $O/run$i/stamps_$t --json $O/run$i/stamps_$t/reading.json > /dev/null || exit 1
    python -c "import json,sys; r=json.load(open('$O/run$i/stamps_$t/reading.json')); print('$t failures', len(r['failures']), [w['reading'][:40] for f in r['failures'] for w in f['waits'][:2]])"
  done
done
