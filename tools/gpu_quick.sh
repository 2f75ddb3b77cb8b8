set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r01k}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu --steps 200 > $O/bench.json 2> $O/bench.err && cut -c1-200 $O/bench.json && python -c "import json; d=json.load(open('$O/bench.json')); print(d['gather_roofline'])"
KB_ITERS=50 timeout -k 10 120 python tools/kbench.py ${KB_NAMES:-fwd_d3 dx_d3 dw_d3 dout_bwd dout_fwd spmm_up0 spmm_up0T spmm_up1 spmm_up1T} > $O/kb.txt 2>&1; cat $O/kb.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --steps 30 --warmup 5 --no-cpu > $O/prof.log 2>&1
python tools/step_timeline.py $(find $O/prof -name '*.db') > $O/timeline.txt; tail -55 $O/timeline.txt
