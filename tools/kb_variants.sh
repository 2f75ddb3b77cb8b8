#!/bin/bash
# Times kbench cases against the product library and each variants/libcfsd_*.so.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/kbv}
rm -rf $OUT; mkdir -p $OUT
export KB_ITERS=${KB_ITERS:-50}
for lib in craniofacialsd-vae_amd/libcfsd.so variants/libcfsd_*.so; do
  echo "== $lib" | tee -a $OUT/all.log
  CFSD_LIB_PATH=$PWD/$lib timeout -k 10 300 python tools/kbench.py ${KB:-fwd_d3} 2>/dev/null | grep " us" | tee -a $OUT/all.log
done
