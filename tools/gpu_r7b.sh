set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r7b
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "bottleneck" > gpurun_out/r7b/bn.log 2>&1 && \
timeout -k 10 1500 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests -m gpu > gpurun_out/r7b/all.log 2>&1
