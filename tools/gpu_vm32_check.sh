set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_vm32.py -v --timeout 120 --timeout-method thread > $O/vm32.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/vm32.log | tail -60; }
tail -3 $O/vm32.log
KB_ITERS=50 timeout -k 10 200 python tools/kbench.py fwd_d3 fwd_d3_vm dx_d3 dxf_d3_vm dw_d3 dw_d3_vm fwd_d2 fwd_d2_vm dx_d2 dxf_d2_vm dw_d2 dw_d2_vm dout_fwd dout_fwd_vm dout_bwd dout_bwd_vm e0_fwd e0_fwd_vm e0_dw e0_dw_vm fwd_e1 fwd_e1_vm dw_e1 dw_e1_vm spmm_up0u spmm_up0_vm spmm_up0T_c spmm_up0T_vm step step_vm > $O/kb.txt 2>&1 || { tail -30 $O/kb.txt; exit 1; }
cat $O/kb.txt
