#!/bin/bash
# A/B the single-GPU launch schedules: bench (K=2000 and K=20) + rocprof kernel durations
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
for sch in classic fused; do
  for rep in 1 2; do
    timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --job-latency 0 --schedule $sch > gpurun_out/ab/$sch.$rep.log 2>&1 || { tail -20 gpurun_out/ab/$sch.$rep.log; exit 1; }
    echo "$sch 2000: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/$sch.$rep.log)"
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --job-latency 0 --schedule $sch > gpurun_out/ab/$sch.k20.$rep.log 2>&1 || exit 1
    echo "$sch 20: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/$sch.k20.$rep.log)"
  done
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/ab/prof_$sch -o run -- python3 bench.py --steps 300 --warmup 20 --job-latency 0 --schedule $sch > gpurun_out/ab/prof_$sch.log 2>&1 || { tail gpurun_out/ab/prof_$sch.log; exit 1; }
done
