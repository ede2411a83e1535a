#!/bin/bash
# Same-box A/B of bench.py flag sets, interleaved per repetition: VARIANTS is a
# '|'-separated list of flag strings ("" = defaults); each runs K=2000 x1 and the driver's
# K=20 W=5 x K20N per rep, REPS reps.  Results append to gpurun_out/ab_flags.txt.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
REPS=${REPS:-3}
IFS='|' read -r -a VS <<< "${VARIANTS:-}"
for rep in $(seq $REPS); do
for v in "${VS[@]}"; do
  a="$(timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --job-latency 0 $v 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1
  b=""; for i in $(seq ${K20N:-2}); do b="$b $(timeout -k 10 120 python bench.py --steps 20 --warmup 5 --job-latency 0 $v 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1; done
  echo "[${v:-defaults}] | K2000: $a | K20:$b" | tee -a gpurun_out/ab_flags.txt
done
done
