set -e
TAG=round6a bash tools/gpu_steps.sh tests
TAG=round6a BENCH_ARGS="--no-cpu" bash tools/gpu_steps.sh bench bench16 prof32
