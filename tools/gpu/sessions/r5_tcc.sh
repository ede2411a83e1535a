#!/bin/bash
# Round 5: L2 (TCC) hit rate per MNIST kernel -- does data written by the previous kernel stay in
# the L2 of the XCD that wrote it across the launch boundary?
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_tcc; mkdir -p $O
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum SQ_WAVES -d $O/p1 -o run --output-format csv -- python3 bench.py --steps 200 --warmup 10 --mode eager --job-latency 0 > $O/log1.txt 2>&1
rc=$?; tail -2 $O/log1.txt; [ $rc = 0 ] || exit $rc
python3 tools/pmc_summary.py $(find $O -name "*counter_collection.csv") > $O/summary.txt && grep -A5 "conv\|fc1\|slab" $O/summary.txt | head -60
find $O -name "*.csv" -size +5M -delete
