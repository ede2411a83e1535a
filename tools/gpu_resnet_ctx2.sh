#!/bin/bash
# ResNet-50 B=256 steady-state kernel trace: where the memsets (fillBuffer) and copy kernels of
# one step sit (the kernels launched around them).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/rctx2; mkdir -p $O /tmp/miopen
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
export MIOPEN_USER_DB_PATH=/tmp/miopen MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/rctx2 -o run --output-format csv -- python3 -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 6 --warmup 3 ${RESNET_ARGS:-} > $O/out.log 2>&1 || { tail -20 $O/out.log; exit 1; }
f=$(find /tmp/rctx2 -name "*kernel_trace.csv" | head -1)
python3 tools/kstats_summary.py --trace "$f" FusedSgd 4 9 > $O/summary.md
python3 tools/trace_context.py "$f" "fillBuffer|copy|Copy|elementwise" FusedSgd 9 > $O/ctx.txt
head -40 $O/summary.md | cut -c1-160; cat $O/ctx.txt | head -150
rm -rf /tmp/rctx2
