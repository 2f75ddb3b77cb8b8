#!/bin/bash
# PMC passes over tools/kbench.py kernels (each pass its own rocprofv3 run, counters only).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/pmc}
KB=${KB:-"fwd_d3 dx_d3 dw_d3"}
rm -rf $OUT; mkdir -p $OUT
export KB_ITERS=${KB_ITERS:-10}
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE" \
         "FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
         "WRITE_SIZE TCC_HIT TCC_MISS TCP_TCC_READ_REQ_LATENCY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "GRBM_TA_BUSY TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_TCC_WRITE_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES SQ_INST_CYCLES_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python tools/kbench.py $KB > $OUT/p$i.log 2>&1
done
echo done
