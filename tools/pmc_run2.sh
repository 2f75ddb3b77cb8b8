#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/pmc2}
KB=${KB:-"fwd_d3 fwd_d3_self"}
mkdir -p $OUT
export KB_ITERS=${KB_ITERS:-10}
i=0
for P in "GRBM_GUI_ACTIVE GRBM_TA_BUSY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
         "TCP_TCP_TA_DATA_STALL_CYCLES TCP_PENDING_STALL_CYCLES TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python tools/kbench.py $KB > $OUT/p$i.log 2>&1
done
echo done
