#!/bin/bash
# Round 3: attention forward 8-wave vs 4-wave (tests + tools/attn_bench.py both variants +
# kernel stats), then the full GPU test suite and the driver's bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3a; mkdir -p $O
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 120 --timeout-method thread > $O/attn_test.log 2>&1 || { echo "attn tests failed"; tail -40 $O/attn_test.log; exit 1; }
tail -1 $O/attn_test.log
for v in 4 8 4 8; do
PTO_ATTN_FWD=$v timeout -k 10 200 python tools/attn_bench.py --impl hip --json-out $O/attn_$v.json > $O/attn_$v.log 2>&1 || { echo "attn bench $v failed"; tail -20 $O/attn_$v.log; exit 1; }
echo "VARIANT fwd=$v $(tail -1 $O/attn_$v.log)"
done
[ -n "$SKIP_SUITE" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; grep -E "PASS|FAIL|ERROR" $O/pytest_gpu.log | tail -5; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_20_5.log; exit 1; }
tail -1 $O/bench_20_5.log
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d /tmp/fprof -o run --output-format csv -- python3 bench.py --steps 2000 --warmup 50 --job-latency 0 > $O/prof_bench.log 2>&1 || { echo "prof failed"; tail -10 $O/prof_bench.log; exit 1; }
f=$(find /tmp/fprof -name "*kernel_stats.csv" | head -1)
python3 tools/kstats_md.py "$f" --top 12 --steps 2050 > $O/kernel_stats.md && cat $O/kernel_stats.md
