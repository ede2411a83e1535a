#!/bin/bash
# GPU-box iteration: numerics tests (incl. GPU e2e job), the HIP worker, bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -m pytorch_operator_amd.harness.mnist --backend rccl --trace --dir gpurun_out/tb > gpurun_out/mnist_hip.log 2>&1 || { echo "worker failed"; tail -30 gpurun_out/mnist_hip.log; exit 1; }
tail -4 gpurun_out/mnist_hip.log
timeout -k 10 300 python bench.py --steps 4000 --warmup 100 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
