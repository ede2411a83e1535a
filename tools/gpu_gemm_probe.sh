#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/gprobe; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
export PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0
timeout -k 10 900 python3 -u tools/gemm_layout_probe.py > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.jsonl
