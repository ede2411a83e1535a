#!/bin/bash
# ResNet-50 bf16 B=256 on one MI355X: 1x1 convs on MIOpen vs as hipBLASLt GEMMs (alternated),
# then a steady-state kernel profile of the GEMM variant.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/rab; mkdir -p $O /tmp/miopen
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
export MIOPEN_USER_DB_PATH=/tmp/miopen MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen
R="python3 -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256"
for r in 1 2; do for c in library gemm; do
timeout -k 10 500 $R --steps 20 --warmup 8 --conv1x1 $c > $O/r_${c}_$r.log 2>&1 || { echo "resnet $c failed"; tail -20 $O/r_${c}_$r.log; exit 1; }
echo "$c $(grep -o '"ms_per_step": [0-9.]*' $O/r_${c}_$r.log)"
done; done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/rprof -o run --output-format csv -- python3 -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 10 --warmup 5 --conv1x1 gemm > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find /tmp/rprof -name "*kernel_trace.csv" | head -1)
python3 tools/kstats_summary.py --trace "$f" FusedSgd 8 15 > $O/summary_gemm.md; head -50 $O/summary_gemm.md; rm -rf /tmp/rprof
