#!/bin/bash
# Same-box A/B: the in-tree library vs every pytorch_operator_amd/_lib/exp/*.so, interleaved
# per repetition (bench K=2000 x1 and the driver's K=20 W=5 x2 per lib per rep; REPS reps).
# Extra bench flags: BENCH_ARGS.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
REPS=${REPS:-3}
for rep in $(seq $REPS); do
for lib in "" $(ls pytorch_operator_amd/_lib/exp/*.so 2>/dev/null); do
  a="$(PTO_HIP_LIB=$lib timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --job-latency 0 $BENCH_ARGS 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1
  b=""; for i in $(seq ${K20N:-2}); do b="$b $(PTO_HIP_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --job-latency 0 $BENCH_ARGS 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1; done
  echo "${lib:-in-tree} | K2000: $a | K20:$b" | tee -a gpurun_out/ab_libs.txt
done
done
