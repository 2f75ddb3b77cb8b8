set -e
TAG=round5y KB_CASES="bneck lin_dec_split latent_bwd lin_enc_pair spmm_up3T" KPROF_ENVS="CFSD_BN_EXP=0;CFSD_BN_EXP=4" bash tools/gpu_steps.sh kprof
