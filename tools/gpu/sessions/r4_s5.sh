#!/bin/bash
# Round 4 session 5: fused fc1+head A/B against the split launches, then the W = 2 x 256
# shared-GPU rehearsal bisected over the round's two step changes (producer push, fused head).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s5; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "fused_tail or on_device" > $O/pytest_tail.log 2>&1; rc=$?; tail -8 $O/pytest_tail.log; [ $rc -ne 0 ] && exit $rc
AB_ENVS="head:PTO_MNIST_FUSE_HEAD=1 tail:PTO_MNIST_FUSE_TAIL=1 tail32:PTO_MNIST_FUSE_TAIL=1,PTO_MNIST_TAIL_REDUCERS=32" bash tools/gpu/ab_libs.sh $O 2 || exit 1
port=29521
for v in "default:" "nopush:PTO_XGMI_PUSH_FC1=0" "unfused:PTO_MNIST_FUSE_HEAD=0"; do
  tag=${v%%:*}; E=${v#*:}
  env $E timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port tools/xgmi_check.py --nblk 256 --out $O/xc_$tag > $O/xc_$tag.log 2>&1
  rc=$?; echo "== xgmi_check nblk 256 $tag rc=$rc"
  python - $O/xc_$tag <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/rank*.json")):
    d = json.load(open(f))
    print({k: d.get(k) for k in ("rank", "all_ok", "kernel_error", "error_after", "push_bit_identical", "graph_in_sync",
                                 "handover_rccl_in_sync", "handover_xgmi_in_sync")})
PY
  case $rc in 0|1) ;; *) exit $rc;; esac
  port=$((port + 1))
done
timeout -k 10 400 python -u -m pytest tests/test_xgmi_emu_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_xgmi_emu.log 2>&1
rc=$?; tail -3 $O/pytest_xgmi_emu.log; [ $rc -ne 0 ] && exit $rc
XAR_KINDS=0 XAR_WORLDS=2,8 XAR_NBLK=128,256 XAR_PUSH=1 timeout -k 10 200 python tools/xgmi_emu_probe.py > $O/xgmi_emu_probe.jsonl 2>$O/xgmi_emu_probe.err
rc=$?; cut -c1-330 $O/xgmi_emu_probe.jsonl; exit $rc
