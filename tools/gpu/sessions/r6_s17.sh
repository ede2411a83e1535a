#!/bin/bash
# round 6: pre-exchange rank barrier on crowded rehearsals (fused form, production kernels) + the
# race's step cross-check; the multi-rank GPU tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s17}; mkdir -p $O
export PYTHONUNBUFFERED=1 PTO_TEST_RECORD_DIR=$O/rec
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests/test_xgmi_gpu.py tests/test_bench_gpu.py tests/test_rccl_gpu.py tests/test_harness.py tests/test_torch_parity_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR" $O/pytest.log | tail -30
[ $rc -ne 0 ] && { grep -E "^E " $O/pytest.log | head -40; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29840 + i)) \
      tools/xgmi_check.py --backend gloo --nblk 256 --stamps --bench --out $O/check$i > $O/check$i.log 2>&1 || { echo "check $i failed"; exit 1; }
  python -c "
import json
d=json.load(open('$O/check$i/rank0.json')); print('$i', d['all_ok'], d['prebarrier'], d['ddp_form'], d['error_after'], d.get('exchange_us'))"
done
