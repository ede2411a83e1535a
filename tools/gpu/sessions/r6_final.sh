#!/bin/bash
# round 6, end of session: the whole GPU suite (records kept), smoke, the driver's bench line x3,
# K=2000 x2, the in-situ step timeline, rocprofv3 kernel stats and the PMC digest of the final tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_final}; mkdir -p $O
export PYTHONUNBUFFERED=1 PTO_TEST_RECORD_DIR=$O/rec
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; grep -E "FAIL|Error" $O/pytest_gpu.log | head; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5_$i.log 2>&1 || { tail -30 $O/bench_20_5_$i.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/bench_20_5_$i.log
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 2000 --warmup 50 --job-latency 0 > $O/bench_2000_$i.log 2>&1 || { tail -30 $O/bench_2000_$i.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/bench_2000_$i.log
done
timeout -k 10 120 python tools/step_timeline.py > $O/timeline.txt 2>&1 || { cat $O/timeline.txt; exit 1; }
grep -E "period|one step|phase times" $O/timeline.txt
bash tools/gpu/profile.sh $O/prof 2050 python3 bench.py --steps 2000 --warmup 50 --job-latency 0 || exit 1
bash tools/gpu/pmc.sh $O/pmc python3 bench.py --steps 200 --warmup 10 --mode eager --job-latency 0 > /dev/null || exit 1
python3 tools/pmc_digest.py $O/pmc/summary.txt conv12_fwd_kernel "void fc1_fwd_kernel<2>" fc1_bwd_head_kernel conv_bwd4_kernel slab_reduce_sgd_kernel > $O/pmc_digest.md && cat $O/pmc_digest.md
