#!/bin/bash
# SQ issue/stall split (one rocprofv3 --pmc pass) + memory-pipeline busy pass over kbench cases.
# usage: KB="dout_bwd dx_d3" OUT=gpurun_out/sq bash tools/pmc_sq.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/sq}
rm -rf $OUT; mkdir -p $OUT
export KB_ITERS=${KB_ITERS:-5}
i=0
for P in "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS TA_TA_BUSY_sum TA_BUSY_sum" \
         "TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_BUSY_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 tools/kbench.py $KB > $OUT/p$i.log 2>&1
done
python tools/pmc_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
