TAG=round5g PYTEST_FILES="tests/test_gpu_unit.py" bash tools/gpu_steps.sh tests
TAG=round5g KB_CASES="fwd_d1_vm fwd_e1_vm fwd_e2_vm fwd_e3_vm fwd_d0" KPROF_ENVS="NONE=0;CFSD_UNIT_FWD=1" bash tools/gpu_steps.sh kprof
