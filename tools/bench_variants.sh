#!/bin/bash
# bench.py (no CPU leg) against the product library and each variants/libcfsd_*.so.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/bv}
rm -rf $OUT; mkdir -p $OUT
for lib in craniofacialsd-vae_amd/libcfsd.so variants/libcfsd_*.so; do
  CFSD_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --steps ${STEPS:-200} > $OUT/one.json 2>/dev/null
  python -c "import json,sys; d=json.load(open('$OUT/one.json')); print('%-45s %9.1f meshes/s  %7.1f us/step' % ('$lib', d['value'], d['ms_per_step']*1e3))" | tee -a $OUT/all.log
done
