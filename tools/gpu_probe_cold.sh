#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/launch
timeout -k 10 200 python tools/cold_start_probe.py > gpurun_out/launch/cold.json 2>gpurun_out/launch/cold.err && cat gpurun_out/launch/cold.json
