cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_ifetch; mkdir -p $O
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d $O/p1 -o run --output-format csv -- python3 bench.py --steps 200 --warmup 10 --mode eager --job-latency 0 > $O/log1.txt 2>&1
rc=$?; tail -3 $O/log1.txt; [ $rc = 0 ] || exit $rc
python3 tools/pmc_summary.py $(find $O -name "*counter_collection.csv") > $O/summary.txt && cat $O/summary.txt | head -80
find $O -name "*.csv" -size +5M -delete
