set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r7a
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_dist.py > gpurun_out/r7a/tests.log 2>&1
