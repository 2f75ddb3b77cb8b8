set -e
timeout -k 10 200 python tools/bn_stamps.py
TAG=round5z PYTEST_FILES="tests/test_gpu_parity.py" PYTEST_K="bottleneck" bash tools/gpu_steps.sh tests
TAG=round5z KB_CASES="bneck lin_dec_split latent_bwd lin_enc_pair spmm_up3T" KPROF_ENVS="CFSD_BN_EXP=0" bash tools/gpu_steps.sh kprof
AB_ENVS="CFSD_FUSE_BOTTLENECK=0;CFSD_FUSE_BOTTLENECK=1" bash tools/ab_bench.sh
