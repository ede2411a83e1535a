#!/bin/bash
# Round-3 attention PMC on the final defaults (8-wave forward, 8-wave LDS-DMA dQ, lean dK/dV
# variant 4, VGPR-form MFMA build): three counter passes, one rocprofv3 run per pass
# (--pmc with --kernel-trace only), then the per-kernel digest.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc4; rm -rf $O; mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_LDS"
P3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE"
i=0
for ctrs in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  cd $R && timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $ctrs -d $O/attn_p$i -o run --output-format csv -- python3 tools/attn_bench.py --impl hip --reps 3 > $O/attn_log$i.txt 2>&1 || { echo "attn pass $i failed"; tail -5 $O/attn_log$i.txt; exit 1; }
  echo "attn pass $i ok"
done
cd $R
python3 tools/pmc_summary.py $(find $O -path "*attn_p*" -name "*counter_collection.csv") > $O/attn_summary.txt
python3 tools/pmc_digest.py $O/attn_summary.txt > $O/attn_digest.md 2>&1 || true
find $O -name "*.csv" -size +5M -delete
cat $O/attn_digest.md | head -30
