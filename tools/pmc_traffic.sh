#!/bin/bash
# HBM traffic per launch of the three D3 conv kernels: FETCH_SIZE and WRITE_SIZE
# in separate rocprofv3 passes (counters only), summarised by tools/pmc_traffic.py
# (gfx950 FETCH x2 correction) into $OUT/<tag>_pmc_traffic_<kernel>.json.
# usage: TAG=r02s OUT=gpurun_out/traffic bash tools/pmc_traffic.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/traffic}
TAG=${TAG:-r02}
rm -rf $OUT; mkdir -p $OUT
export KB_ITERS=${KB_ITERS:-10}
CASES=${CASES:-"fwd_d3:conv_fwd_mfma<32, 32, 1, 9>:conv_fwd_d3 dx_d3:conv_dx_mfma<32, 32, 9>:conv_dx_d3 dw_d3:conv_dw_mfma<32, 32>:conv_dw_d3"}
# bf16: CASES="fwd_d3_b16:conv_fwd_b16<32, 32, 1, unsigned short>:conv_fwd_d3_bf16 ..."
IFS=$'\n'
for case in $(echo "$CASES" | sed 's/ \([A-Za-z0-9_]*:\)/\n\1/g'); do
  kb=${case%%:*}; rest=${case#*:}; pat=${rest%%:*}; name=${rest#*:}
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$kb/pmc_fetch -o run -- python3 tools/kbench.py $kb > $OUT/$kb.fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$kb/pmc_write -o run -- python3 tools/kbench.py $kb > $OUT/$kb.write.log 2>&1
  python tools/pmc_traffic.py $OUT/$kb "$pat" > $OUT/${TAG}_pmc_traffic_${name}.json
  cat $OUT/${TAG}_pmc_traffic_${name}.json
done
