#!/bin/bash
# Counter evidence for the coarse chain (levels 2-4 + bottleneck): SQ issue /
# stall split + memory pipeline (tools/pmc_sq.sh passes) and HBM traffic
# (FETCH_SIZE / WRITE_SIZE, tools/pmc_traffic.sh) of the coarse kernels.
# usage: TAG=r04a OUT=gpurun_out/coarse bash tools/gpu_coarse_pmc.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/coarse}
KB="${KB:-fwd_d0 dx_d0 dw_d0 fwd_d1 pair_d1 lin_enc_fwd lin_dec_fwd lin_dec_dx}" OUT=$OUT/sq bash tools/pmc_sq.sh
CASES="fwd_d0:conv_fwd_lat<64, 64, 1, 2>:conv_fwd_d0 dx_d0:conv_dx_lat<64, 64, 2>:conv_dx_d0 pair_d1:conv_bwd_lat_pair<64, 32, 2>:conv_pair_d1 fwd_d1:conv_fwd_mfma<64, 32, 1, 3>:conv_fwd_d1" \
  TAG=${TAG:-r04} OUT=$OUT/traffic bash tools/pmc_traffic.sh
