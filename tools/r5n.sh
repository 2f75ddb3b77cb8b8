set -e
timeout -k 10 120 ./tools/mfma_wave_probe.bin | tee gpurun_out/round5n_probe.txt
TAG=round5n KB_CASES="fwd_d3_vm" KPROF_ENVS="CFSD_VM32_FWD_EXP=6;CFSD_VM32_FWD_EXP=14;CFSD_VM32_FWD_EXP=30;CFSD_VM32_FWD_EXP=30 CFSD_VM32_FWD_GRID=1024" bash tools/gpu_steps.sh kprof
