#!/bin/bash
# PMC passes (one rocprofv3 run per counter set, counters + kernel trace only) over
# tools/kbench.py cases; summary per kernel into $OUT/summary.txt.
# usage: KB="fwd_d3 dx_d3" OUT=gpurun_out/pmc bash tools/pmc_kernels.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/pmc}
KB=${KB:-"fwd_d3 dx_d3 dw_d3"}
rm -rf $OUT; mkdir -p $OUT
export KB_ITERS=${KB_ITERS:-5}
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 tools/kbench.py $KB > $OUT/p$i.log 2>&1
done
python tools/pmc_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
