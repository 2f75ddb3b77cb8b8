set -e
TAG=round6c PYTEST_FILES="tests/test_gpu_parity.py" PYTEST_K="reduce or fused or slab or deferred" bash tools/gpu_steps.sh tests
TAG=round6c BENCH_ARGS="--no-cpu" bash tools/gpu_steps.sh bench prof32
