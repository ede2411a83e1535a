#!/bin/bash
# Round 5: kernel stats (stream-launched bench, K = 2000) and the PMC digest (three counter
# passes over the eager bench) of the five-launch MNIST step, plus the in-situ timeline.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r5_prof}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/step_timeline.py --json $O/timeline.json > $O/timeline.txt 2>&1 || { cat $O/timeline.txt; exit 1; }
grep -E "period|one step" $O/timeline.txt
bash tools/gpu/profile.sh $O/prof 2050 python3 bench.py --steps 2000 --warmup 50 --job-latency 0 || exit 1
bash tools/gpu/pmc.sh $O/pmc python3 bench.py --steps 200 --warmup 10 --mode eager --job-latency 0 > $O/pmc_run.log 2>&1 || { tail -20 $O/pmc_run.log; exit 1; }
cp $O/pmc/summary.txt $O/pmc_summary.txt
python3 tools/pmc_digest.py $O/pmc_summary.txt > $O/pmc_digest_table.md && cat $O/pmc_digest_table.md
