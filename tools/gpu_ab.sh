#!/bin/bash
# A/B schedule variants in one GPU session
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
python -c "from pytorch_operator_amd.ops import _native; _native.build()" || exit 1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for args in "--overlap 1" "--overlap 0" "--overlap 0 --fuse-conv12 1" "--overlap 1 --mode eager" "--overlap 0 --mode eager"; do
  echo "== $args"
  timeout -k 10 120 python bench.py --steps 3000 --warmup 100 $args 2>&1 | grep -v amdgpu.ids | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['config']['exec'])" || exit 1
done
