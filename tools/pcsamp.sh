#!/bin/bash
# Stochastic PC sampling of tools/kbench.py cases (stall reasons per instruction).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/pcs}
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/list.txt 2>&1 || true
grep -i -A12 "pc.sampl\|PC_SAMPL" $OUT/list.txt | head -60
export KB_ITERS=${KB_ITERS:-20}
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-stochastic} --pc-sampling-unit ${UNIT:-cycles} --pc-sampling-interval ${INTERVAL:-65536} --output-format csv -d $OUT/run -o pcs -- python tools/kbench.py ${KB:-fwd_d3} > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
ls -R $OUT/run | head
