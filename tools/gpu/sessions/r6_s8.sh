#!/bin/bash
# round 6: the start-up race with the round-5 forms as candidates (rccl-r5, xgmi-r5)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s8}; mkdir -p $O
export PYTHONUNBUFFERED=1 PTO_TEST_RECORD_DIR=$O/rec
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests/test_bench_gpu.py tests/test_rccl_gpu.py tests/test_xgmi_gpu.py tests/test_harness.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR" $O/pytest.log | tail -30
[ $rc -ne 0 ] && { grep -E "^E " $O/pytest.log | head -40; exit 1; }
for i in 1 2; do
  PTO_XGMI_ANY_BACKEND=1 timeout -k 10 240 python bench.py --gpus 2 --backend gloo --allreduce auto --steps 400 --warmup 40 --job-latency 0 > $O/bench_w2_auto_$i.log 2>&1 || { tail -30 $O/bench_w2_auto_$i.log; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/bench_w2_auto_$i.log') if l.startswith('{\"metric')][-1]); print(d['ms_per_step'], d['replicas_in_sync'], d['config']['allreduce_trial'])"
done
