#!/bin/bash
# A/B libraries: builds libcfsd.so as of other git revisions into variants/
# (git-ignored), for ab_kernel.sh / kb_variants.sh / bench_variants.sh.
# usage: bash tools/build_variants.sh name:rev [name:rev ...]
#   e.g. bash tools/build_variants.sh prev:HEAD~1 r03:r03-tag
# (Kernel geometry is compiled in as constants; variants are revisions, not -D switches.)
set -e
cd "$(dirname "$0")/.."
mkdir -p variants
for v in "$@"; do
  name=${v%%:*}; rev=${v#*:}
  tmp=/tmp/var_$name
  rm -rf $tmp && mkdir -p $tmp
  git archive "$rev" craniofacialsd-vae_amd/csrc include | tar -x -C $tmp
  make -C $tmp/craniofacialsd-vae_amd/csrc -j8 > $tmp/build.log 2>&1
  cp $tmp/craniofacialsd-vae_amd/libcfsd.so variants/libcfsd_$name.so
  echo built $name from $rev
done
