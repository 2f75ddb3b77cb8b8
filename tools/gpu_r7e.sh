# role split of the coarse pair kernels (events + kernel-trace stats)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
KB="pair_d0_vm dx_d0 dw_d0 pair_d1_vm dx_d1 dw_d1 rowsub_e1_vm dgonly_e1_vm dw_e1_vm rowsub_e2_vm fwd_d1_vm fwd_d0_up fwd_e1_vm bneck" OUT=gpurun_out/r7e bash tools/kb_prof.sh
