set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03l
timeout -k 10 300 python -u -m pytest tests/test_gpu_vm32.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r03l/vm32.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r03l/vm32.log | head -20; tail -5 gpurun_out/r03l/vm32.log; exit 1; }
tail -2 gpurun_out/r03l/vm32.log
KB="fwd_d3_vm fwd_d2_vm" KB_ITERS=30 OUT=gpurun_out/kbv4 timeout -k 10 400 bash tools/kb_variants.sh 2>&1 | tail -12
