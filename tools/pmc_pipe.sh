#!/bin/bash
# Memory-pipeline PMC passes (TA / TD / TCP / TCC busy and stall counters), one
# rocprofv3 run per pass, over tools/kbench.py cases; summary per kernel.
# usage: KB="fwd_d3 dout_fwd" OUT=gpurun_out/pipe bash tools/pmc_pipe.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/pipe}
KB=${KB:-"fwd_d3"}
rm -rf $OUT; mkdir -p $OUT
export KB_ITERS=${KB_ITERS:-5}
i=0
for P in "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
         "TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum" \
         "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_REQUEST_sum" \
         "TCC_BUSY_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 tools/kbench.py $KB > $OUT/p$i.log 2>&1
done
python tools/pmc_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
