#!/bin/bash
# Device time (rocprofv3 kernel trace, avg per dispatch) of kbench cases
# against the product library and each variants/libcfsd_*.so.  (Eager
# event timing of a kbench loop is host-bound below ~15 us per launch.)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/kbv}
rm -rf $OUT; mkdir -p $OUT
export KB_ITERS=${KB_ITERS:-50}
for lib in craniofacialsd-vae_amd/libcfsd.so variants/libcfsd_*.so; do
  v=$(basename $lib .so)
  [ -f "$lib" ] || continue
  echo "== $lib" | tee -a $OUT/all.log
  CFSD_LIB_PATH=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o kb -- python3 tools/kbench.py ${KB:-fwd_d3} > $OUT/$v.log 2>&1
  python tools/prof_summary.py $(find $OUT/$v -name '*.db' | head -1) 40 | grep cfsd | cut -c1-140 | tee -a $OUT/all.log
done
