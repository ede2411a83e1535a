#!/bin/bash
# A/B: the in-tree library vs every pytorch_operator_amd/_lib/exp/*.so (bench K=2000 x3, K=20 x2)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
for lib in "" $(ls pytorch_operator_amd/_lib/exp/*.so 2>/dev/null); do
  a=""; for i in 1 2 3; do a="$a $(PTO_HIP_LIB=$lib timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --job-latency 0 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1; done
  b=""; for i in 1 2; do b="$b $(PTO_HIP_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --job-latency 0 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1; done
  echo "${lib:-in-tree} | K2000:$a | K20:$b"
done
done
