set -e
TAG=round5w PYTEST_FILES="tests/test_gpu_parity.py" PYTEST_K="bottleneck" bash tools/gpu_steps.sh tests
AB_ENVS="CFSD_FUSE_BOTTLENECK=0;CFSD_FUSE_BOTTLENECK=1" bash tools/ab_bench.sh
TAG=round5w bash tools/gpu_steps.sh prof32
