#!/bin/bash
# A/B of whole-step execution on one MI355X: hipGraph replay (spg <= warm-up) vs the
# captured kernel list launched onto the stream; new GPU tests; Llama-3 8B with the
# residual-fused RMSNorm.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/lab; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_llm_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do for l in graph stream; do
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --job-latency 0 --launch $l > $O/b20_${l}_$r.log 2>&1 || { echo "bench $l failed"; tail -20 $O/b20_${l}_$r.log; exit 1; }
echo "k20 $l $(grep -o '"ms_per_step": [0-9.]*' $O/b20_${l}_$r.log)"
done; done
for l in graph stream; do
timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --job-latency 0 --launch $l > $O/b2000_$l.log 2>&1 || { echo "bench $l failed"; tail -20 $O/b2000_$l.log; exit 1; }
echo "k2000 $l $(grep -o '"ms_per_step": [0-9.]*' $O/b2000_$l.log)"
done
timeout -k 10 400 python -u -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4 --steps 6 --warmup 3 > $O/llama.log 2>&1 || { echo "llama failed"; tail -20 $O/llama.log; exit 1; }
grep '"metric"' $O/llama.log
