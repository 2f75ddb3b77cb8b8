# fp32 vertex-major vs batch-major: tests, bench lines, kernel stats + timelines of both layouts.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03e}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_vm32.py -v --timeout 120 --timeout-method thread > $O/vm32.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/vm32.log | tail -40; }
tail -2 $O/vm32.log
for L in vm bm; do
  F=""; [ $L = bm ] && F="--batch-major"
  timeout -k 10 200 python bench.py --no-cpu --no-extras --steps 2000 $F > $O/bench_$L.json 2> $O/bench_$L.err || { tail -20 $O/bench_$L.err; exit 1; }
  cut -c1-330 $O/bench_$L.json; echo
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$L -o bench -- python3 bench.py --steps 30 --warmup 5 --no-cpu --no-extras $F > $O/prof_$L.log 2>&1 || { tail -20 $O/prof_$L.log; exit 1; }
  python tools/step_timeline.py $(find $O/prof_$L -name '*.db' | head -1) > $O/timeline_$L.txt
  python tools/prof_summary.py $(find $O/prof_$L -name '*.db' | head -1) 45 > $O/kernel_stats_$L.txt
done
tail -48 $O/timeline_vm.txt
# locality experiment: the same vertex-major kernels on an RCM-relabelled topology
KBN="fwd_d3_vm dxf_d3_vm dw_d3_vm fwd_d2_vm dxf_d2_vm dw_d2_vm dout_fwd_vm dout_bwd_vm spmm_up0_vm spmm_up0T_vm fwd_d3 dx_d3 dw_d3"
for R in 0 1; do
  if [ $R = 1 ]; then export KB_REORDER=1; else unset KB_REORDER; fi
  KB_ITERS=30 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kbprof_$R -o kb -- python3 tools/kbench.py $KBN > $O/kbprof_$R.log 2>&1 || { tail -20 $O/kbprof_$R.log; exit 1; }
  python tools/prof_summary.py $(find $O/kbprof_$R -name '*.db' | head -1) 30 > $O/kb_stats_reorder$R.txt
  echo "== reorder $R"; cat $O/kb_stats_reorder$R.txt
done
