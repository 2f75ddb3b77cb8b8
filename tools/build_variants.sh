#!/bin/bash
# Experimental timing variants of libcfsd.so (macro switches), into variants/ (git-ignored).
set -e
cd "$(dirname "$0")/../craniofacialsd-vae_amd/csrc"
mkdir -p ../../variants
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950"
for v in "$@"; do
  name=${v%%:*}; defs=${v#*:}
  mkdir -p /tmp/var_$name
  for f in spiral_conv spiral_conv_bf16 spiral_conv_vm16 spiral_conv_vm32 pool_swap train_ops; do
    $H $F $defs -c $f.hip -o /tmp/var_$name/$f.o &
  done
  wait
  $H -shared --offload-arch=gfx950 -o ../../variants/libcfsd_$name.so /tmp/var_$name/*.o
  echo built $name
done
