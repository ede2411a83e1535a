#!/bin/bash
# Round-end readiness on one MI355X: the GPU tests (PYTEST_SEL, default all of tests/), smoke(),
# the driver's bench line, and (unless SKIP_PROF) a rocprofv3 kernel-stats table of the bench.
#   bash tools/gpu/check.sh [OUT_DIR]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/check}; mkdir -p $O
export PYTHONUNBUFFERED=1
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest ${PYTEST_SEL:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_20_5.log; exit 1; }
tail -1 $O/bench_20_5.log
[ -n "$SKIP_PROF" ] && exit 0
bash tools/gpu/profile.sh $O/prof 2050 python3 bench.py --steps 2000 --warmup 50 --job-latency 0
