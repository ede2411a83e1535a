#!/bin/bash
# round 6: the crowded 2 x 256 rehearsal three times with exchange stamps (stops at the first failure)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s16}; mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29820 + i)) \
      tools/xgmi_check.py --backend gloo --nblk 256 --stamps --out $O/check$i > $O/check$i.log 2>&1
  rc=$?
  python -c "
import json,glob
for f in sorted(glob.glob('$O/check$i/rank*.json')):
    d=json.load(open(f)); print('$i', f[-10:], d.get('all_ok'), d.get('error_after'), [ (d.get(k) or {}).get('xgmi_crosscheck') for k in ('handover_rccl_times','handover_xgmi_times')], d.get("handover_xgmi_error"), d.get("prebarrier"))
"
  [ $rc -ne 0 ] && { echo "run $i rc=$rc"; grep -h "Error" $O/check$i.log | tail -3; python tools/xgmi_stamps.py $O/check$i/stamps_main 2>&1 | tail -20; exit 1; }
done
exit 0
