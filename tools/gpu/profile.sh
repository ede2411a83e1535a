#!/bin/bash
# rocprofv3 kernel trace + stats of one command; prints the kernel-stats table
# (tools/kstats_md.py, per-step figures when STEPS > 0).
#   bash tools/gpu/profile.sh OUT_DIR STEPS python3 bench.py --steps 2000 --warmup 50 --job-latency 0
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$1; STEPS=$2; shift 2; mkdir -p $O
timeout -s KILL ${PROF_TIMEOUT:-240} rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- "$@" > $O/prof.log 2>&1 || { echo "prof failed"; tail -10 $O/prof.log; exit 1; }
f=$(find $O/raw -name "*kernel_stats.csv" | head -1)
python3 tools/kstats_md.py "$f" --top ${TOP:-12} --steps $STEPS > $O/kernel_stats.md && cat $O/kernel_stats.md
find $O/raw -name "*.csv" -size +20M -delete
