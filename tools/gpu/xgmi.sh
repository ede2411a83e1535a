#!/bin/bash
# xGMI exchange on one box: the W = 2/4/8 emulation tests and latency probe (one launch, all
# emulated ranks on the GPU), then the multi-process rehearsal (ranks sharing the GPU, gloo
# reference collectives) at each WORLDS x NBLKS, and a 2-rank xGMI bench.
#   WORLDS="2 4" NBLKS="0 256" bash tools/gpu/xgmi.sh OUT_DIR
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/xgmi}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_xgmi_emu_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_emu.log 2>&1
rc=$?; tail -3 $O/pytest_emu.log; [ $rc -ne 0 ] && exit $rc
XAR_KINDS=${XAR_KINDS:-0} XAR_WORLDS=${XAR_WORLDS:-2,8} XAR_NBLK=${XAR_NBLK:-128,256} timeout -k 10 200 python tools/xgmi_emu_probe.py > $O/emu_probe.jsonl 2>$O/emu_probe.err
rc=$?; cat $O/emu_probe.jsonl; [ $rc -ne 0 ] && { tail -20 $O/emu_probe.err; exit $rc; }
port=29640
for W in ${WORLDS:-2 4}; do for NB in ${NBLKS:-0}; do
  port=$((port + 1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port $port \
    tools/xgmi_check.py --backend gloo --nblk $NB --bench --out $O/check_w${W}_nblk$NB > $O/check_w${W}_nblk$NB.log 2>&1
  rc=$?; echo "== xgmi_check W=$W nblk=$NB rc=$rc"; grep -h '^{' $O/check_w${W}_nblk$NB.log | cut -c1-400
  case $rc in 0) ;; 1) FAILED=1;; *) exit $rc;; esac
done; done
[ -n "$FAILED" ] && exit 1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((port + 1)) \
  bench.py --gpus 2 --backend gloo --allreduce xgmi --steps 400 --warmup 40 > $O/bench_w2.log 2>&1 || { echo "xgmi bench failed"; tail -40 $O/bench_w2.log; exit 1; }
tail -1 $O/bench_w2.log
