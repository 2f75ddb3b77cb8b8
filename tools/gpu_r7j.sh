# Round-6 checkpoint at HEAD: full GPU suite, smoke, default bench (fp32 + bf16 block),
# fp32 / bf16 step timelines, kernel stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r7j}; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --steps 30 --warmup 5 --no-cpu --no-extras > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
python tools/step_timeline.py $(find $O/prof -name '*.db' | head -1) > $O/timeline_fp32.txt; tail -1 $O/timeline_fp32.txt
python tools/prof_summary.py $(find $O/prof -name '*.db' | head -1) 60 > $O/kernel_stats_fp32.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof16 -o bench -- python3 bench.py --steps 30 --warmup 5 --no-cpu --no-extras --precision bf16 > $O/prof16.log 2>&1 || { tail -30 $O/prof16.log; exit 1; }
python tools/step_timeline.py $(find $O/prof16 -name '*.db' | head -1) > $O/timeline_bf16.txt; tail -1 $O/timeline_bf16.txt
python tools/prof_summary.py $(find $O/prof16 -name '*.db' | head -1) 60 > $O/kernel_stats_bf16.txt
