set -e
TAG=round5v1 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_roofline.py" PYTEST_K="bottleneck or fused_reduce or priced or adam_scaled" bash tools/gpu_steps.sh tests
AB_ENVS="CFSD_FUSE_BOTTLENECK=0;CFSD_FUSE_BOTTLENECK=1" bash tools/ab_bench.sh
TAG=round5v bash tools/gpu_steps.sh prof32
