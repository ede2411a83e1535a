#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/launch
timeout -k 10 120 python tools/launch_overhead_probe.py > gpurun_out/launch/default.json 2>gpurun_out/launch/err0.log && cat gpurun_out/launch/default.json
