#!/bin/bash
# round 6: fc1 bias folded into the first split-K partial (fc1_bwd_head / head_kernel stop
# reloading b1) -- kernel + parity tests, A/B against the previous tree (abtree/head), PMC digest
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s21}; mkdir -p $O
export PYTHONUNBUFFERED=1
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_torch_parity_gpu.py tests/test_rccl_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TL_ARGS="--by-mod fc1_bwd_head:216" bash tools/gpu/ab_trees.sh $O/ab 2 || exit 1
bash tools/gpu/pmc.sh gpurun_out/r6_s21/pmc python3 bench.py --steps 200 --warmup 10 --mode eager --job-latency 0 || exit 1
python3 tools/pmc_digest.py gpurun_out/r6_s21/pmc/summary.txt conv12_fwd_kernel conv_bwd4_kernel fc1_bwd_head_kernel slab_reduce_sgd_kernel "void fc1_fwd_kernel<2>" > $O/pmc_digest.md && cat $O/pmc_digest.md
