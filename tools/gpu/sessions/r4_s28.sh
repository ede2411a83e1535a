#!/bin/bash
# Round 4 session 28 (end of round): readiness (GPU tests, smoke, bench line) and a kernel-stats
# profile of the Llama-3 8B step with this round's attention kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
SKIP_PROF=1 bash tools/gpu/check.sh gpurun_out/r4s28/check || exit 1
PROF_TIMEOUT=400 TOP=25 bash tools/gpu/profile.sh gpurun_out/r4s28/llama_prof 5 python3 -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 4 --steps 5 --warmup 2 --zero 0 || exit 1
