#!/bin/bash
# Round 4 session 4: fc1+head fused launch (numerics, timeline, A/B vs the split launches),
# the producer-pushed dW_fc1 xGMI exchange (emulation at W = 2/8 x 128/256, bit-identity,
# latency probe), the W = 2 shared-GPU rehearsal at nblk 256.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s4; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "fc1_head or fused_head" > $O/pytest_fused_head.log 2>&1
rc=$?; tail -12 $O/pytest_fused_head.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_kernels.log 2>&1
rc=$?; tail -3 $O/pytest_kernels.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_xgmi_emu_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_xgmi_emu.log 2>&1
rc=$?; tail -25 $O/pytest_xgmi_emu.log; [ $rc -ne 0 ] && exit $rc
XAR_KINDS=0 XAR_WORLDS=2,8 XAR_NBLK=128,256 XAR_PUSH=0,1 timeout -k 10 200 python tools/xgmi_emu_probe.py > $O/xgmi_emu_probe.jsonl 2>$O/xgmi_emu_probe.err
rc=$?; cat $O/xgmi_emu_probe.jsonl; [ $rc -ne 0 ] && { tail -20 $O/xgmi_emu_probe.err; exit $rc; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
  tools/xgmi_check.py --nblk 256 --out $O/xgmi_check_w2_nblk256 > $O/xgmi_check_w2_nblk256.log 2>&1
rc=$?; grep -h '"rank"' $O/xgmi_check_w2_nblk256.log | cut -c1-600; [ $rc -ne 0 ] && { tail -30 $O/xgmi_check_w2_nblk256.log; exit $rc; }
AB_ENVS="unfused:PTO_MNIST_FUSE_HEAD=0" bash tools/gpu/ab_libs.sh $O 2
