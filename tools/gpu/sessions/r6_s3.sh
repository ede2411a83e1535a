#!/bin/bash
# round 6: LDS bank-conflict-free layouts in conv12_fwd / fc1_bwd_head (tools/lds_banks_fwd.py):
# numerics tests, same-box A/B against the round-5 kernels (exp/r5.so), PMC digest of the new step
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s3}; mkdir -p $O
export PYTHONUNBUFFERED=1
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_torch_parity_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "^E |FAIL|Error" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/ab_libs.sh $O/ab 2 || exit 1
bash tools/gpu/pmc.sh $O/pmc python3 bench.py --steps 200 --warmup 10 --mode eager --job-latency 0 > $O/pmc_run.log 2>&1 || { tail -20 $O/pmc_run.log; exit 1; }
head -20 $O/pmc/summary.txt
