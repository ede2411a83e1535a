#!/bin/bash
# PMC counters per kernel (kernel-trace only; no sys/runtime trace with --pmc)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R && python -c "from pytorch_operator_amd.ops import _native; _native.build()" || exit 1
rm -rf $R/gpurun_out/pmc; mkdir -p $R/gpurun_out/pmc
i=0
for ctrs in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAIT_ANY" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  cd $R && timeout -k 10 240 rocprofv3 --kernel-trace --pmc $ctrs -d $R/gpurun_out/pmc/p$i -o run --output-format csv -- python3 bench.py --steps 200 --warmup 10 --mode eager --job-latency 0 > $R/gpurun_out/pmc/log$i.txt 2>&1 || { tail -5 $R/gpurun_out/pmc/log$i.txt; exit 1; }
done
find $R/gpurun_out/pmc -name "*.csv" | head -20
python3 tools/pmc_summary.py $(find $R/gpurun_out/pmc -name "*counter_collection.csv") > $R/gpurun_out/pmc/summary.txt && head -5 $R/gpurun_out/pmc/summary.txt
