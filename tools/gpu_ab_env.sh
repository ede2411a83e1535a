#!/bin/bash
# A/B of HIP runtime knobs on the 1-GPU bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 4000 --warmup 100 > gpurun_out/ab_base_$i.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_base_$i.log
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python bench.py --steps 4000 --warmup 100 > gpurun_out/ab_kernarg_$i.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_kernarg_$i.log
done
