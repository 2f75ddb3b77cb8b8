# vm32 tests + fp32/bf16 bench lines + fp32 step timeline (quick iteration loop).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03h}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_vm32.py ${EXTRA_TESTS} -q -x --timeout 120 --timeout-method thread > $O/vm32.log 2>&1 || { grep -E "FAIL|Error|assert|error" $O/vm32.log | head -30; tail -5 $O/vm32.log; exit 1; }
tail -2 $O/vm32.log
timeout -k 10 200 python bench.py --no-cpu --no-extras --steps 2000 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json; echo
timeout -k 10 200 python bench.py --precision bf16 --no-cpu --no-extras --steps 2000 > $O/bench_bf16.json 2> $O/bench_bf16.err || { tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-200 $O/bench_bf16.json; echo
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --steps 30 --warmup 5 --no-cpu --no-extras > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python tools/step_timeline.py $(find $O/prof -name '*.db' | head -1) > $O/timeline.txt
python tools/prof_summary.py $(find $O/prof -name '*.db' | head -1) 45 > $O/kernel_stats.txt
rm -rf $O/prof
grep -E "bwd_out|out_small|recon_lap|swap|conv_fwd_in|dw_in|kernel-sum" $O/timeline.txt
