set -e
CFSD_VM32_FWD_PIPE=1 TAG=round5j PYTEST_FILES="tests/test_gpu_vm32.py" PYTEST_K="fwd" bash tools/gpu_steps.sh tests
TAG=round5j KB_CASES="fwd_d3_vm fwd_d2_vm" KPROF_ENVS="CFSD_VM32_FWD_PIPE=0;CFSD_VM32_FWD_PIPE=1;CFSD_VM32_FWD_PIPE=0;CFSD_VM32_FWD_PIPE=1" bash tools/gpu_steps.sh kprof
for c in fwd_d3_vm_self fwd_d3_vm_shift; do
TAG=round5j KB_CASES="$c" KPROF_ENVS="CFSD_VM32_FWD_PIPE=0;CFSD_VM32_FWD_PIPE=1" bash tools/gpu_steps.sh kprof
done
