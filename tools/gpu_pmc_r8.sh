# Round-6 close: fresh HBM-traffic PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs) for the
# kernels bench.py's roofline blocks price -- fp32 D3 dx (flat), bf16 D3 pair -- plus the D3 forwards
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r8r}; rm -rf $O; mkdir -p $O
CASES="dxf_d3_vm:conv_dx_flat_vm32<32, 32, 16, float>:conv_dx_d3_vm fwd_d3_vm:conv_fwd_vm32<32, 32, 1, 2, 1>:conv_fwd_d3_vm" OUT=$O/traffic TAG=$TAG bash tools/pmc_traffic.sh
CASES="pair_d3_b16:conv_bwd_vm16_pair<16>:conv_pair_d3_bf16_vm fwd_d3_b16:conv_fwd_vm16<32, 32, 1, unsigned short>:conv_fwd_d3_bf16_vm" OUT=$O/traffic16 TAG=$TAG bash tools/pmc_traffic.sh
