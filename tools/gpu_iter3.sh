#!/bin/bash
# kernel numerics tests, the lib A/B (tools/gpu_ab_libs.sh), then one PMC pass of LDS counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu > gpurun_out/kt3.log 2>&1; rc=$?
tail -3 gpurun_out/kt3.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh || exit 1
rm -rf gpurun_out/pmc_lds
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/pmc_lds -o run --output-format csv -- python3 bench.py --steps 200 --warmup 10 --mode eager --job-latency 0 > gpurun_out/pmc_lds.log 2>&1 || exit 1
python3 tools/pmc_summary.py $(find gpurun_out/pmc_lds -name "*counter_collection.csv") > gpurun_out/pmc_lds.txt && grep -A4 "conv\|fc1\|head\|slab" gpurun_out/pmc_lds.txt
