#!/bin/bash
# round 6: the 96-VGPR exchange (one phase-2 batch per thread) -- the production kernels beside a
# spinning 256-workgroup exchange (profiles/r6_xgmi_geometry.md), exchange latency, world-2 benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s9}; mkdir -p $O
export PYTHONUNBUFFERED=1 PTO_TEST_RECORD_DIR=$O/rec
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_xgmi_gpu.py tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR" $O/pytest.log | tail -40
[ $rc -ne 0 ] && { grep -E "^E " $O/pytest.log | head -40; exit 1; }
port=29750
for NB in 128 256; do
  port=$((port + 1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port \
    tools/xgmi_check.py --backend gloo --nblk $NB --bench --stamps --out $O/check_nblk$NB > $O/check_nblk$NB.log 2>&1
  rc=$?; echo "== xgmi_check W=2 nblk=$NB rc=$rc"; grep -h '^{' $O/check_nblk$NB.log | cut -c1-900
  [ $rc -ne 0 ] && exit 1
done
for form in 0 1; do
  PTO_DDP_FUSED=$form PTO_XGMI_ANY_BACKEND=1 timeout -k 10 240 python bench.py --gpus 2 --backend gloo --allreduce xgmi --steps 400 --warmup 40 --job-latency 0 > $O/bench_w2_xgmi_f$form.log 2>&1 || { echo "bench w2 xgmi f$form failed"; tail -30 $O/bench_w2_xgmi_f$form.log; exit 1; }
  echo "w2 xgmi fused=$form: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_w2_xgmi_f$form.log) $(grep -o '"replicas_in_sync": [a-z]*' $O/bench_w2_xgmi_f$form.log)"
done
