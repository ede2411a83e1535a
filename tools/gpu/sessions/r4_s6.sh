#!/bin/bash
# Round 4 session 6: start-up latency (1-replica job in the bench line, 2-pod job via the bench
# GPU test, recorded), flash-attention dK/dV chain-ahead variant A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s6; mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_job_$i.json 2>$O/bench_job_$i.err || { tail -20 $O/bench_job_$i.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('create_to_first_step_s'), json.dumps(d['job'].get('startup_breakdown')))" $O/bench_job_$i.json
done
PTO_TEST_RECORD_DIR=$GRAFT_REPO_ROOT/$O timeout -k 10 900 python -u -m pytest tests/test_bench_gpu.py -x -v --timeout 400 --timeout-method thread > $O/pytest_bench.log 2>&1
rc=$?; tail -5 $O/pytest_bench.log; [ $rc -ne 0 ] && exit $rc
for f in $O/bench_w2_*.json; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d.get('create_to_first_step_s'), json.dumps(d['job'].get('startup_breakdown')))" $f; done
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread -k "dkdv" > $O/pytest_attn.log 2>&1
rc=$?; tail -3 $O/pytest_attn.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for v in 4 5; do
  PTO_ATTN_DKDV=$v timeout -k 10 200 python tools/attn_bench.py --impl hip --json-out $O/attn_dkdv${v}_$rep.json > $O/attn_dkdv${v}_$rep.log 2>&1 || { tail -20 $O/attn_dkdv${v}_$rep.log; exit 1; }
  echo "dkdv $v rep $rep: $(tail -1 $O/attn_dkdv${v}_$rep.log)"
done; done
bash tools/gpu/ab_libs.sh $O/ab 2 || exit 1
bash tools/gpu/profile.sh $O/prof 2050 python3 bench.py --steps 2000 --warmup 50 --job-latency 0 || exit 1
bash tools/gpu/pmc.sh $O/pmc python3 bench.py --steps 200 --warmup 10 --mode eager --job-latency 0 || exit 1
timeout -k 10 120 python tools/step_timeline.py --json $O/timeline.json > $O/timeline.txt 2>&1 || { cat $O/timeline.txt; exit 1; }
grep -E "period|one step" $O/timeline.txt
