#!/bin/bash
# round 6: the fused DDP forms (RCCL: 6 launches + one all-reduce; xGMI: 5 launches, fc gradients
# computed in the exchange) -- numerics tests, the xGMI rehearsal, world-2 and forced world-1
# benches before (PTO_DDP_FUSED=0) / after
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s6}; mkdir -p $O
export PYTHONUNBUFFERED=1 PTO_TEST_RECORD_DIR=$O/rec
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_torch_parity_gpu.py tests/test_rccl_gpu.py tests/test_xgmi_gpu.py ${EXTRA_TESTS} -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  grep -E "PASS|FAIL|ERROR" $O/pytest.log | tail -40
  [ $rc -ne 0 ] && { grep -E "^E " $O/pytest.log | head -40; exit 1; }
fi
port=29700
for NB in 0 256; do
  port=$((port + 1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port \
    tools/xgmi_check.py --backend gloo --nblk $NB --out $O/check_nblk$NB > $O/check_nblk$NB.log 2>&1
  rc=$?; echo "== xgmi_check W=2 nblk=$NB rc=$rc"; grep -h '^{' $O/check_nblk$NB.log | cut -c1-600
  [ $rc -ne 0 ] && exit 1
done
for form in 0 1; do for ar in rccl xgmi; do
  PTO_DDP_FUSED=$form timeout -k 10 240 python bench.py --gpus 2 --backend gloo --allreduce $ar --steps 400 --warmup 40 --job-latency 0 > $O/bench_w2_${ar}_f$form.log 2>&1 || { echo "bench w2 $ar f$form failed"; tail -30 $O/bench_w2_${ar}_f$form.log; exit 1; }
  echo "w2 $ar fused=$form: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_w2_${ar}_f$form.log) $(grep -o '"replicas_in_sync": [a-z]*' $O/bench_w2_${ar}_f$form.log)"
done; done
for form in 0 1; do
  PTO_DDP_FUSED=$form timeout -k 10 240 python bench.py --gpus 1 --backend nccl --force-collectives 1 --steps 400 --warmup 40 --job-latency 0 > $O/bench_w1_forced_f$form.log 2>&1 || { echo "forced bench f$form failed"; tail -30 $O/bench_w1_forced_f$form.log; exit 1; }
  echo "w1 forced fused=$form: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_w1_forced_f$form.log) $(grep -o '"rccl_ms_per_step": [0-9.]*' $O/bench_w1_forced_f$form.log) $(grep -o '"rccl_graph_ms_per_step": [0-9.]*' $O/bench_w1_forced_f$form.log)"
done
