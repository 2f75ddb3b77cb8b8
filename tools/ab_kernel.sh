#!/bin/bash
# A/B of one kernel's average duration: kernel-trace stats of `kbench.py $KB` under the
# product library and each variants/libcfsd_*.so, same box, same process layout.
# usage (from gpurun): KB=step PAT=dw_reduce bash tools/ab_kernel.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/ab}
rm -rf $OUT; mkdir -p $OUT
export KB_ITERS=${KB_ITERS:-30}
for rep in 1 2; do
  for lib in craniofacialsd-vae_amd/libcfsd.so variants/libcfsd_*.so; do
    name=$(basename $lib .so)_$rep
    CFSD_LIB_PATH=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$name -o run \
      -- python3 tools/kbench.py ${KB:-step} > $OUT/$name.log 2>&1
    python3 tools/prof_summary.py $(find $OUT/$name -name '*.db' | head -1) 200 | grep -E "${PAT:-.}" | sed "s|^|$name |" || true
    rm -rf $OUT/$name
  done
done
