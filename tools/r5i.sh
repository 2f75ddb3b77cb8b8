TAG=round5i KB_CASES="fwd_d3_vm fwd_d3_vm_self fwd_d3_vm_shift fwd_d3_vm_noact fwd_d3_vm_x2 dxf_d3_vm dw_d3_vm" bash tools/gpu_steps.sh kprof
