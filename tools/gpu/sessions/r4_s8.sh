#!/bin/bash
# Round 4 session 8: conv_bwd4 split groups with software-pipelined 2a / 2b operand reads vs the
# unpipelined split (same box), kernel tests, then the final default's kernel stats + PMC digest.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s8; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_kernels.log 2>&1
rc=$?; tail -3 $O/pytest_kernels.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_libs.sh $O/ab 2 || exit 1
bash tools/gpu/profile.sh $O/prof 2050 python3 bench.py --steps 2000 --warmup 50 --job-latency 0 || exit 1
bash tools/gpu/pmc.sh $O/pmc python3 bench.py --steps 200 --warmup 10 --mode eager --job-latency 0 > $O/pmc_run.log 2>&1 || { tail -20 $O/pmc_run.log; exit 1; }
cp $O/pmc/summary.txt $O/pmc_summary.txt && wc -l $O/pmc_summary.txt
