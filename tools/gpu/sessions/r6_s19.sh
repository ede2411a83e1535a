#!/bin/bash
# round 6: conv_bwd4 LDS bank conflicts (un-pool store swizzle, xn row stride 30) -- kernel tests,
# same-box A/B against the committed kernels (exp/head.so), PMC digest of the new step
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s19}; mkdir -p $O
export PYTHONUNBUFFERED=1
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_torch_parity_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TL_ARGS="--by-mod conv_bwd4:4" bash tools/gpu/ab_libs.sh $O/ab 2 || exit 1
bash tools/gpu/pmc.sh gpurun_out/r6_s19/pmc python3 bench.py --steps 200 --warmup 10 --mode eager --job-latency 0 || exit 1
python3 tools/pmc_digest.py gpurun_out/r6_s19/pmc > $O/pmc_digest.md 2>&1 && cat $O/pmc_digest.md
