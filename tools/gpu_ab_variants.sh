# Kernel + whole-step A/B of the product library against every variants/libcfsd_*.so (same box).
# usage: KB="pair_d1_vm" PAT="pair" AB_ARGS="--precision bf16" bash tools/gpu_ab_variants.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-abv}; mkdir -p $O
OUT=$O/abk bash tools/ab_kernel.sh > $O/abk.txt 2>&1 || { tail -20 $O/abk.txt; exit 1; }
cat $O/abk.txt
ENVS="NONE=0"
for lib in variants/libcfsd_*.so; do ENVS="$ENVS;CFSD_LIB_PATH=$PWD/$lib"; done
AB_ENVS="$ENVS" bash tools/ab_bench.sh > $O/abb.txt 2>&1 || { tail -20 $O/abb.txt; exit 1; }
cat $O/abb.txt
if [ -n "$AB16" ]; then
  AB_ARGS="--precision bf16" AB_ENVS="$ENVS" bash tools/ab_bench.sh > $O/abb16.txt 2>&1 || { tail -20 $O/abb16.txt; exit 1; }
  cat $O/abb16.txt
fi
