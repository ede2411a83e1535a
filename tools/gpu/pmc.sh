#!/bin/bash
# PMC digest of one command: three counter passes (one rocprofv3 run each, --pmc with
# --kernel-trace only, within the per-block counter limits), summarised per kernel by
# tools/pmc_summary.py into OUT_DIR/summary.txt.
#   bash tools/gpu/pmc.sh OUT_DIR python3 bench.py --steps 200 --warmup 10 --mode eager --job-latency 0
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/$1; shift; rm -rf $O; mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_LDS"
P3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE"
i=0
for ctrs in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  cd $R && timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $ctrs -d $O/p$i -o run --output-format csv -- "$@" > $O/log$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $O/log$i.txt; exit 1; }
  echo "pass $i ok"
done
cd $R
python3 tools/pmc_summary.py $(find $O -name "*counter_collection.csv") > $O/summary.txt && head -40 $O/summary.txt
find $O -name "*.csv" -size +5M -delete
