# bf16 step (vertex-major level 0/1): bench line + kernel stats + step timeline.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03f}; mkdir -p $O
timeout -k 10 200 python bench.py --precision bf16 --no-cpu --no-extras --steps 2000 > $O/bench_bf16.json 2> $O/bench_bf16.err || { tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-300 $O/bench_bf16.json; echo
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_bf16 -o bench -- python3 bench.py --precision bf16 --steps 30 --warmup 5 --no-cpu --no-extras > $O/prof_bf16.log 2>&1 || { tail -20 $O/prof_bf16.log; exit 1; }
python tools/step_timeline.py $(find $O/prof_bf16 -name '*.db' | head -1) > $O/timeline_bf16.txt
python tools/prof_summary.py $(find $O/prof_bf16 -name '*.db' | head -1) 45 > $O/kernel_stats_bf16.txt
rm -rf $O/prof_bf16
cat $O/timeline_bf16.txt
