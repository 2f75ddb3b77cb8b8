# Round evidence: all GPU tests, default bench line (fp32, with CPU baseline), bf16 bench,
# kernel stats + step timelines (fp32, bf16), D3 FETCH/WRITE traffic of the kernels the step runs.
# usage (via gpurun): TAG=r03k bash tools/gpu_evidence.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03k}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json; echo
timeout -k 10 300 python bench.py --precision bf16 --no-cpu --no-extras --steps 2000 > $O/bench_bf16.json 2> $O/bench_bf16.err || { tail -30 $O/bench_bf16.err; exit 1; }
cut -c1-300 $O/bench_bf16.json; echo
for P in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$P -o bench -- python3 bench.py --precision $P --steps 30 --warmup 5 --no-cpu --no-extras > $O/prof_$P.log 2>&1 || { tail -30 $O/prof_$P.log; exit 1; }
  python tools/step_timeline.py $(find $O/prof_$P -name '*.db' | head -1) > $O/timeline_$P.txt
  python tools/prof_summary.py $(find $O/prof_$P -name '*.db' | head -1) 45 > $O/kernel_stats_$P.txt
  rm -rf $O/prof_$P
  tail -1 $O/timeline_$P.txt
done
CASES="fwd_d3_vm:conv_fwd_vm32<32, 32, 1, 2, 1>:conv_fwd_d3_vm dxf_d3_vm:conv_dx_flat_vm32<32, 32, 16>:conv_dx_d3_vm dw_d3_vm:conv_dw_vm32:conv_dw_d3_vm" OUT=$O/traffic TAG=$TAG bash tools/pmc_traffic.sh > /dev/null
CASES="fwd_d3_b16:conv_fwd_vm16<32, 32, 1, unsigned short>:conv_fwd_d3_bf16_vm dxf_d3_b16:conv_dx_flat_vm16<32, 32, unsigned short, 16>:conv_dx_d3_bf16_vm dw_d3_b16:conv_dw_vm16<unsigned short>:conv_dw_d3_bf16_vm" OUT=$O/traffic16 TAG=$TAG bash tools/pmc_traffic.sh > /dev/null
cat $O/traffic/*.json $O/traffic16/*.json
