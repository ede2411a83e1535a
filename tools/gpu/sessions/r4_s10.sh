#!/bin/bash
# Round 4 session 10: the multi-process xGMI tests after the graph-launch hand-over change,
# smoke(), the driver's bench line, and per-kernel times of the attention backward passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s10; mkdir -p $O
export PYTHONUNBUFFERED=1
PYTEST_SEL=tests/test_xgmi_gpu.py SKIP_PROF=1 bash tools/gpu/check.sh $O/check || exit 1
PROF_TIMEOUT=200 TOP=8 bash tools/gpu/profile.sh $O/attn_prof 0 python3 tools/attn_bench.py --impl hip --reps 10 || exit 1
