set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03j
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -q -x -k "flat or train or graph" --timeout 120 --timeout-method thread > gpurun_out/r03j/bf16.log 2>&1 || { tail -30 gpurun_out/r03j/bf16.log; exit 1; }
tail -2 gpurun_out/r03j/bf16.log
KB="dxf_d3_b16 fwd_d3_b16 dw_d3_b16" KB_ITERS=30 OUT=gpurun_out/kb3 timeout -k 10 300 bash tools/kb_prof.sh 2>&1 | grep -E "cfsd|us$" | head -12
KB="fwd_d3_vm dxf_d3_vm dw_d3_vm dout_bwd_flat" OUT=gpurun_out/sq3 timeout -k 10 400 bash tools/pmc_sq.sh > /dev/null 2>&1 || true
grep -A30 "conv_fwd_vm32\|conv_dx_flat_vm32\|conv_dw_mfma\|conv_bwd_out_vm" gpurun_out/sq3/summary.txt | grep -E "^[a-z_v]|GRBM|SQ_WAVE_CYCLES|SQ_WAIT_ANY|SQ_WAIT_INST_ANY|SQ_ACTIVE_INST_ANY|SQ_VALU_MFMA|SQ_INSTS_MFMA|TA_BUSY|TD_TD|TCC_BUSY|TCC_HIT|TCC_MISS|SQ_INSTS_VMEM_RD|SQ_WAVES" | head -80
