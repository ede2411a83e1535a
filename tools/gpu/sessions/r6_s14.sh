#!/bin/bash
# round 6: diagnose the xgmi-r5 cross-check at W=2 (bench auto race record)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s14}; mkdir -p $O
export PYTHONUNBUFFERED=1
PTO_XGMI_ANY_BACKEND=1 timeout -k 10 240 python bench.py --gpus 2 --backend gloo --allreduce auto --steps 100 --warmup 20 --job-latency 0 > $O/bench.log 2>&1; rc=$?
grep -v '^{"metric' $O/bench.log | tail -5
python -c "
import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{\"metric')][-1]); print(json.dumps(d['config']['allreduce_trial'], indent=1))"
exit $rc
