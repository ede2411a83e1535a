#!/bin/bash
# round 6: the automatic pre-exchange barrier (XgmiAllReduce.crowded) -- the multi-rank GPU tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s20}; mkdir -p $O
export PYTHONUNBUFFERED=1 PTO_TEST_RECORD_DIR=$O/rec
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests/test_xgmi_gpu.py tests/test_bench_gpu.py tests/test_harness.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR" $O/pytest.log | tail -30
[ $rc -ne 0 ] && { grep -E "^E " $O/pytest.log | head -40; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29871 \
  bench.py --gpus 4 --backend gloo --allreduce auto --steps 200 --warmup 20 --job-latency 0 > $O/bench_w4.log 2>&1 || { tail -30 $O/bench_w4.log; exit 1; }
python -c "
import json; d=json.loads([l for l in open('$O/bench_w4.log') if l.startswith('{\"metric')][-1]); t=d['config']['allreduce_trial']; print(d['ms_per_step'], d['replicas_in_sync'], d['grad_allreduce_error'], {k:v for k,v in t.items() if 'ms_per' in k or k in ('picked','xgmi_crosscheck')})"
