TAG=round5h PYTEST_FILES="tests/test_gpu_vm32.py" bash tools/gpu_steps.sh tests
TAG=round5h KB_CASES="fwd_d3_vm fwd_d2_vm" bash tools/gpu_steps.sh kprof
TAG=round5h BENCH_ARGS="--no-cpu" bash tools/gpu_steps.sh bench
