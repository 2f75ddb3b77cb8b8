# RCCL capture tests, repeated (thread-local capture mode)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r7k; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_configs.py -k rccl > $O/rccl_$i.log 2>&1 || { grep -E "Error|error|what|Exception" $O/rccl_$i.log | head -30; exit 1; }
  tail -1 $O/rccl_$i.log
done
