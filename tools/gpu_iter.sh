#!/bin/bash
# quick GPU iteration: kernel tests, phase profile, bench, rocprof stats
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
python -c "from pytorch_operator_amd.ops import _native; _native.build(verbose=False)" || exit 1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/phase_profile.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/phase.log || exit 1
timeout -k 10 180 python bench.py --steps 2000 --warmup 50 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench.log || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof; mkdir -p $R/gpurun_out/prof
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run -- python3 bench.py --steps 500 --warmup 20 --mode eager > $R/gpurun_out/prof/bench.log 2>&1 || { tail -5 $R/gpurun_out/prof/bench.log; exit 1; }
python tools/rocpd_summary.py $(find $R/gpurun_out/prof -name "*.db" | head -1)
