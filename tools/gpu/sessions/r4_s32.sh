#!/bin/bash
# Round 4 session 32: the xGMI rehearsals after moving the shared-GPU 256-workgroup hand-over
# stage onto a 128-workgroup exchange (tests/test_xgmi_gpu.py, three times).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s32; mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py -x -q --timeout 300 --timeout-method thread -k "allreduce_ranks" > $O/pytest_xgmi_$i.log 2>&1 || { tail -30 $O/pytest_xgmi_$i.log; exit 1; }
  echo "run $i: $(tail -1 $O/pytest_xgmi_$i.log)"
done
