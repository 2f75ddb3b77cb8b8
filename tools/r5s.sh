set -e
TAG=round5s KB_CASES="dout_bwd_flat dout_bwd_flat_b16" KPROF_ENVS="NONE=0;CFSD_BWDOUT_BPC=2;CFSD_BWDOUT_BPC=3;CFSD_BWDOUT_BPC=5;CFSD_BWDOUT_BPC=6" bash tools/gpu_steps.sh kprof
TAG=round5s BENCH_ARGS="--no-cpu" bash tools/gpu_steps.sh bench bench16
