#!/bin/bash
# Round 4 session 33 (final): readiness on the final tree (GPU tests, smoke, bench line).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
SKIP_PROF=1 bash tools/gpu/check.sh gpurun_out/r4s33/check
