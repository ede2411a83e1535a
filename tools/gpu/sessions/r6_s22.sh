#!/bin/bash
# round 6: host cost per launch, hipLaunchKernel vs hipModuleLaunchKernel (tools/dbg/launch_api_probe.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_s22}; mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2; do
  timeout -k 10 300 python tools/dbg/launch_api_probe.py --reps 9 > $O/probe_$i.json 2> $O/probe_$i.err || { tail -20 $O/probe_$i.err; exit 1; }
  cat $O/probe_$i.json
done
