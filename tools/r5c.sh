TAG=round5c PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_roofline.py tests/test_gpu_train_driver.py tests/test_gpu_vm32.py" PYTEST_K="fused_reduce or dist or roofline or train or graph or step or generate or refused" BENCH_ARGS="--no-cpu --no-extras" bash tools/gpu_steps.sh tests bench prof32 bench16
TAG=round5c bash tools/dp_timeline.sh
