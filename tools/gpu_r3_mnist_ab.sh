#!/bin/bash
# Round-3 MNIST step A/B on one box: in-tree vs exp/*.so variant libraries (tools/build_exp.sh),
# then bench flag variants on the in-tree library.  Lines go to gpurun_out/ab_libs.txt.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
REPS=${REPS:-2} bash tools/gpu_ab_libs2.sh || exit 1
for rep in 1 2; do
for fl in "--fc-sgd tail" "--fc-sgd next"; do
  a="$(timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --job-latency 0 $fl 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1
  b=""; for i in 1 2; do b="$b $(timeout -k 10 120 python bench.py --steps 20 --warmup 5 --job-latency 0 $fl 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1; done
  echo "flags[$fl] | K2000: $a | K20:$b" | tee -a gpurun_out/ab_libs.txt
done
done
