set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r01i; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu --steps 100 > $O/bench.json 2> $O/bench.err && cat $O/bench.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --steps 30 --warmup 5 --no-cpu > $O/prof.log 2>&1
python tools/step_timeline.py $(find $O/prof -name '*.db') > $O/timeline.txt; tail -75 $O/timeline.txt
