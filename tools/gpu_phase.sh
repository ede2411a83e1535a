#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python tools/phase_profile.py > gpurun_out/phase.txt 2>&1 || { tail -20 gpurun_out/phase.txt; exit 1; }
cat gpurun_out/phase.txt
