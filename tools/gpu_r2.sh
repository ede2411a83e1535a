#!/bin/bash
# Round-2 GPU iteration: GPU tests, driver-contract bench runs (incl. the create->first-step
# job through the operator), a long bench, and a rocprofv3 kernel-trace of graph replays.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
STAGE=${1:-all}
if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_20_5.log 2>&1 || { echo "bench 20/5 failed"; tail -30 gpurun_out/bench_20_5.log; exit 1; }
  tail -1 gpurun_out/bench_20_5.log
  for i in 1 2; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --job-latency 0 > gpurun_out/bench_20_5_nl$i.log 2>&1 || { echo "bench failed"; exit 1; }
    tail -1 gpurun_out/bench_20_5_nl$i.log | cut -c1-200
  done
  timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --job-latency 0 > gpurun_out/bench_2000.log 2>&1 || { echo "bench 2000 failed"; tail -30 gpurun_out/bench_2000.log; exit 1; }
  tail -1 gpurun_out/bench_2000.log | cut -c1-200
fi
if [ "$STAGE" = all ] || [ "$STAGE" = prof ]; then
  mkdir -p gpurun_out/prof_r2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2 -o run -- python3 bench.py --steps 200 --warmup 20 --job-latency 0 > gpurun_out/prof_r2/bench.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_r2/bench.log; exit 1; }
  find gpurun_out/prof_r2 -name "*stats*"
fi
