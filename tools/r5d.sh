TAG=round5d KB_CASES="fwd_d0_up fwd_d1_vm fwd_e1_vm" KPROF_ENVS="NONE=0;CFSD_PT_GRID=2;CFSD_PT_GRID=3" bash tools/gpu_steps.sh kprof
TAG=round5d PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_dist.py" PYTEST_K="fused_reduce or dist" BENCH_ARGS="--no-cpu --no-extras" bash tools/gpu_steps.sh tests bench prof32 bench16 prof16
TAG=round5d bash tools/dp_timeline.sh
