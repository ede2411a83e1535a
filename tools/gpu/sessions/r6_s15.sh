#!/bin/bash
# round 6: diagnose the step cross-check in the crowded 2 x 256 rehearsal
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s15}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29811 \
    tools/xgmi_check.py --backend gloo --nblk 256 --stamps --out $O/check > $O/check.log 2>&1
rc=$?; echo "rc=$rc"; grep -h "Error\|error" $O/check.log | grep -v amdgpu.ids | tail -5
python -c "
import json,glob
for f in sorted(glob.glob('$O/check/rank*.json')):
    d=json.load(open(f)); print(f, d.get('error_after'), d.get('kernel_error'))
    for k in ('handover_rccl_times','handover_xgmi_times'):
        t=d.get(k) or {}; print(k, t.get('xgmi_crosscheck'), t.get('xgmi_skipped'), t.get('picked'))
"
ls $O/check
exit 0
