#!/bin/bash
# Round 3: xGMI emulation probe with the chunked slab vs per-sample slab (W=2/8), and the
# world-2 RCCL-path split step graph replay vs native stream launch (gloo on one GPU).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
XAR_KINDS=0 XAR_WORLDS=2,8 XAR_NBLK=128,256 XAR_SLAB=chunk,sample timeout -k 10 300 python -u tools/xgmi_emu_probe.py > gpurun_out/r3_xgmi_emu_probe.jsonl 2> gpurun_out/r3_xgmi_emu_probe.err || { echo "emu probe failed"; tail -20 gpurun_out/r3_xgmi_emu_probe.err; exit 1; }
cat gpurun_out/r3_xgmi_emu_probe.jsonl
REPS=2 timeout -k 10 600 bash tools/gpu_split_ab.sh || exit 1
