# bf16 evidence pass: C5-shaped bench line, bf16 kernel stats, bf16 D3 PMC traffic.
# usage (via gpurun): TAG=r03a bash tools/gpu_bf16_evidence.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03}; mkdir -p $O
timeout -k 10 400 python bench.py --precision bf16 --augmented 50000 --steps 2000 --warmup 50 --no-cpu --no-extras > $O/bench_c5_bf16.json 2> $O/bench_c5.err || { tail -30 $O/bench_c5.err; exit 1; }
cut -c1-300 $O/bench_c5_bf16.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bf16 -o bench -- python3 bench.py --precision bf16 --steps 30 --warmup 5 --no-cpu --no-extras > $O/prof_bf16.log 2>&1 || { tail -30 $O/prof_bf16.log; exit 1; }
python tools/step_timeline.py $(find $O/prof_bf16 -name '*.db' | head -1) > $O/timeline_bf16.txt; tail -8 $O/timeline_bf16.txt
python tools/prof_summary.py $(find $O/prof_bf16 -name "*.db" | head -1) 40 > $O/kernel_stats_bf16.txt
CASES="fwd_d3_b16:conv_fwd_b16<32, 32, 1, unsigned short>:conv_fwd_d3_bf16 dx_d3_b16:conv_dx_b16<32, 32, unsigned short>:conv_dx_d3_bf16 dw_d3_b16:conv_dw_b16<32, 32, unsigned short>:conv_dw_d3_bf16" OUT=$O/traffic TAG=$TAG bash tools/pmc_traffic.sh
