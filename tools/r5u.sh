set -e
TAG=round5u bash tools/gpu_steps.sh tests
TAG=round5u KB_CASES="fwd_d3_vm fwd_d3_vm_noact fwd_d2_vm" bash tools/gpu_steps.sh kprof
TAG=round5u BENCH_ARGS="--no-cpu" bash tools/gpu_steps.sh bench bench16
