#!/bin/bash
# Round 4 session 7: split-group conv_bwd4 (now the default) numerics + wave-priority A/B for
# its group A; start-up with the dataset drawn by this library's kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s7; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_kernels.log 2>&1
rc=$?; tail -3 $O/pytest_kernels.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_job_$i.json 2>$O/bench_job_$i.err || { tail -20 $O/bench_job_$i.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('create_to_first_step_s'), json.dumps(d['job'].get('startup_breakdown')))" $O/bench_job_$i.json
done
bash tools/gpu/ab_libs.sh $O/ab 2 || exit 1
