C="fwd_d0_up pair_d0_vm fwd_d1_vm pair_d1_vm fwd_e1_vm rowsub_e1_vm fwd_e2_vm fwd_e3_vm rowsub_e2_vm rowsub_e3_vm spmm_up1T_vm spmm_up2T_vm spmm_up3T_vm lin_dec_split latent_bwd lin_enc_pair lin_enc_fwd_vm"
O=gpurun_out/round5b; mkdir -p $O
timeout -k 10 120 ./tools/mfma_power_probe.bin > $O/mfma_power_probe.txt 2>&1 && cat $O/mfma_power_probe.txt
TAG=round5b KB_CASES="$C red_items" SQ_CASES="$C" bash tools/gpu_steps.sh kbench sq pmc32 pmc16
