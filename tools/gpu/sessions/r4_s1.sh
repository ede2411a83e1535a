#!/bin/bash
# Round 4 session 1: any-order launch probe, kernel numerics after the prune, in-situ step
# timeline, bench K=2000 / K=20, kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s1; mkdir -p $O
export PYTHONUNBUFFERED=1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o $O/anyorder_probe tools/probes/anyorder_probe.hip || exit 1
timeout -k 10 60 $O/anyorder_probe > $O/anyorder.jsonl 2>&1; echo "probe rc=$?"; cat $O/anyorder.jsonl
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_kernels.log 2>&1
rc=$?; tail -5 $O/pytest_kernels.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python tools/step_timeline.py --json $O/timeline.json > $O/timeline.txt 2>&1 || { cat $O/timeline.txt; exit 1; }
cat $O/timeline.txt
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --job-latency 0 > $O/bench2000_$i.json 2>$O/bench_err.log || exit 1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --job-latency 0 > $O/bench20_$i.json 2>>$O/bench_err.log || exit 1
done
grep -ho '"ms_per_step": [0-9.]*' $O/bench*.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 2000 --warmup 50 --job-latency 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs head -12
