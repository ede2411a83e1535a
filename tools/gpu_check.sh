#!/bin/bash
# One GPU-box session: kernel tests, smoke, short bench (each step time-limited).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 420 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 180 python bench.py --steps 2000 --warmup 50 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
timeout -k 10 180 python bench.py --steps 500 --warmup 20 --mode eager > gpurun_out/bench_eager.log 2>&1 || { tail -30 gpurun_out/bench_eager.log; exit 1; }
cat gpurun_out/bench_eager.log
timeout -k 10 180 python bench.py --steps 300 --warmup 20 --kernels torch > gpurun_out/bench_torch.log 2>&1 || { tail -30 gpurun_out/bench_torch.log; exit 1; }
cat gpurun_out/bench_torch.log
