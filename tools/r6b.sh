set -e
TAG=round6b KB_CASES="dxf_d3_vm dxf_d2_vm" KPROF_ENVS="CFSD_DX32_PD=2;CFSD_DX32_PD=1;CFSD_DX32_PD=3;CFSD_DX32_PD=4;CFSD_DX32_PD=2" bash tools/gpu_steps.sh kprof
