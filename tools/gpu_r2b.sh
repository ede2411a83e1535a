#!/bin/bash
# Round-2 re-entry check on one MI355X: every GPU test, smoke, the headline bench at the
# driver's settings and at K=2000, Llama-3 8B (HIP flash attention vs SDPA) and ResNet-50.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r2b
O=gpurun_out/r2b
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_20_5.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_20_5.log; exit 1; }
tail -1 $O/bench_20_5.log
timeout -k 10 300 python bench.py --job-latency 0 > $O/bench_def.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_def.log; exit 1; }
tail -1 $O/bench_def.log
for a in auto sdpa; do
timeout -k 10 600 python -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4 --steps 6 --warmup 3 --attn $a > $O/llama8b_$a.log 2>&1 || { echo "llama8b failed"; tail -20 $O/llama8b_$a.log; exit 1; }
tail -1 $O/llama8b_$a.log
done
timeout -k 10 420 python -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256 --steps 20 --warmup 8 > $O/resnet50.log 2>&1 || { echo "resnet failed"; tail -20 $O/resnet50.log; exit 1; }
tail -1 $O/resnet50.log
