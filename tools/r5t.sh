set -e
TAG=round5t PYTEST_FILES="tests/test_gpu_dist.py tests/test_gpu_parity.py tests/test_gpu_vm32.py" PYTEST_K="dist or adam or vm or fused or step" bash tools/gpu_steps.sh tests
TAG=round5t bash tools/gpu_steps.sh prof32 prof16
