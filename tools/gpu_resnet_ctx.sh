#!/bin/bash
# ResNet-50 B=256 steady-state kernel trace: per-family summary + where the slow elementwise
# kernels sit in the step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/rctx; mkdir -p $O /tmp/miopen
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
export MIOPEN_USER_DB_PATH=/tmp/miopen MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen
timeout -k 10 500 python3 -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 5 --warmup 3 > $O/find.log 2>&1 || { tail -20 $O/find.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/find.log
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/rctx -o run --output-format csv -- python3 -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 6 --warmup 3 > $O/out.log 2>&1 || { tail -20 $O/out.log; exit 1; }
f=$(find /tmp/rctx -name "*kernel_trace.csv" | head -1)
python3 tools/kstats_summary.py --trace "$f" FusedSgd 4 9 > $O/summary.md
python3 tools/trace_context.py "$f" "elementwise|vectorized|direct_copy|copy" FusedSgd 9 20 > $O/elementwise.txt
head -30 $O/summary.md; head -80 $O/elementwise.txt
rm -rf /tmp/rctx
