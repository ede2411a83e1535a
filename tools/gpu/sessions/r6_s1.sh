#!/bin/bash
# round 6, first GPU session: the self-launching bench, RCCL rank count, torch-parity tests,
# then the driver-shaped bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6_s1; mkdir -p $O
export PYTHONUNBUFFERED=1 PTO_TEST_RECORD_DIR=$O/rec
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_torch_parity_gpu.py tests/test_bench_gpu.py -k "parity or contract or self_launch or nranks or bench_configuration or torch_ddp" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest.log | tail -20
[ $rc -ne 0 ] && { tail -60 $O/pytest.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20_$i.json 2>> $O/bench_err.txt || { tail -30 $O/bench_err.txt; exit 1; }
  tail -1 $O/bench_k20_$i.json | cut -c1-400
done
