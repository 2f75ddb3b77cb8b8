set -e
TAG=round6f KB_CASES="spmm_up0T_vm spmm_up0T_vm_rcm" bash tools/gpu_steps.sh kprof
CASES="spmm_up0T_vm_rcm:spmm_sched_csr_k:spmm_up0T_vm_rcm" OUT=gpurun_out/round6f/traffic TAG=round6f bash tools/pmc_traffic.sh > /dev/null
cat gpurun_out/round6f/traffic/*.json
AB_ENVS="CFSD_UPT_RCM=0;CFSD_UPT_RCM=1" bash tools/ab_bench.sh
