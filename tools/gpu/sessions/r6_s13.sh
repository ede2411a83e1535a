#!/bin/bash
# round 6: the xGMI candidates' start-up step cross-check against RCCL (autotune.crosscheck_step)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s13}; mkdir -p $O
export PYTHONUNBUFFERED=1 PTO_TEST_RECORD_DIR=$O/rec
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests/test_bench_gpu.py tests/test_xgmi_gpu.py tests/test_rccl_gpu.py tests/test_harness.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR" $O/pytest.log | tail -30
[ $rc -ne 0 ] && { grep -E "^E " $O/pytest.log | head -40; exit 1; }
python -c "
import json,glob
for f in sorted(glob.glob('$O/rec/bench_w2_*.json')):
    d=json.load(open(f)); t=d['config'].get('allreduce_trial'); print(f.split('/')[-1], d['ms_per_step'], t and t.get('xgmi_crosscheck'), t and t.get('picked'))
"
