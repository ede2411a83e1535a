#!/bin/bash
# Round-3 step A/B on one MI355X: numerics of the new kernels, per-kernel phase profile, then
# bench.py over the schedule knobs (K=2000 x2 and the driver's K=20 W=5 x2 per variant).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_xgmi_emu_gpu.py > gpurun_out/r3_kt.log 2>&1; rc=$?
  grep -E "passed|failed|PASS|FAIL|Error" gpurun_out/r3_kt.log | tail -40
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 180 python tools/phase_profile.py > gpurun_out/r3_phase.txt 2>&1 || { tail -20 gpurun_out/r3_phase.txt; exit 1; }
cat gpurun_out/r3_phase.txt | grep -v amdgpu.ids
VARIANTS=${VARIANTS:-"--conv-chunk=1 --fc-sgd=tail --stage=0|--conv-chunk=4 --fc-sgd=tail --stage=0|--conv-chunk=4 --fc-sgd=fused --stage=0|--conv-chunk=4 --fc-sgd=fused --stage=1|--conv-chunk=4 --fc-sgd=fused --stage=1 --store-fc-grads=0"}
IFS='|' read -ra VS <<< "$VARIANTS"
for rep in 1 2; do
for v in "${VS[@]}"; do
  a=""; for i in 1 2; do a="$a $(timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --job-latency 0 $v 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1; done
  b=""; for i in 1 2; do b="$b $(timeout -k 10 120 python bench.py --steps 20 --warmup 5 --job-latency 0 $v 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1; done
  echo "[$v] | K2000:$a | K20:$b" | tee -a gpurun_out/r3_ab.txt
done
done
