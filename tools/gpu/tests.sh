#!/bin/bash
# One or more GPU test files (optionally a -k expression), each under its own time limit.
#   bash tools/gpu/tests.sh OUT_DIR "k-expression or empty" tests/test_a_gpu.py [tests/test_b_gpu.py ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$1; K=$2; shift 2; mkdir -p $O
export PYTHONUNBUFFERED=1
for f in "$@"; do
  n=$(basename $f .py)
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $f -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/$n.log 2>&1
  rc=$?; grep -E "passed|failed|error" $O/$n.log | tail -1; [ $rc -ne 0 ] && { tail -40 $O/$n.log; exit $rc; }
done
exit 0
