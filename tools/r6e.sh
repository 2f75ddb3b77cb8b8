set -e
TAG=round6e PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_vm32.py" PYTEST_K="trainstep or graph" bash tools/gpu_steps.sh tests
AB_ENVS="CFSD_STEPS_PER_GRAPH=2;CFSD_STEPS_PER_GRAPH=8;CFSD_STEPS_PER_GRAPH=16" bash tools/ab_bench.sh
