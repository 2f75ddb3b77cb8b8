#!/bin/bash
# A/B of kbench cases in the template's vertex order vs the RCM locality order
# (kernel-trace device times), for the product library and each variants/*.so.
# usage: KB="fwd_d3 dx_d3" bash tools/reorder_ab.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/reorder}
rm -rf $OUT; mkdir -p $OUT
export KB_ITERS=${KB_ITERS:-30}
for lib in craniofacialsd-vae_amd/libcfsd.so variants/libcfsd_*.so; do
  v=$(basename $lib .so)
  [ -f "$lib" ] || continue
  for mode in orig rcm; do
    if [ $mode = rcm ]; then export KB_REORDER=1; else unset KB_REORDER; fi
    CFSD_LIB_PATH=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v-$mode -o kb -- python3 tools/kbench.py $KB > $OUT/$v-$mode.log 2>&1
    echo "== $v $mode"
    python tools/prof_summary.py $(find $OUT/$v-$mode -name '*.db' | head -1) 40 | grep cfsd | cut -c1-150
  done
done
