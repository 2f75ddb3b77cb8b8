# Round 7 evidence pass: default bench (fp32 line + bf16 block), fp32 / bf16
# step timelines, SQ counters of the coarse chain at HEAD.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r7c}; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --steps 30 --warmup 5 --no-cpu --no-extras > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
python tools/step_timeline.py $(find $O/prof -name '*.db' | head -1) > $O/timeline_fp32.txt; tail -3 $O/timeline_fp32.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof16 -o bench -- python3 bench.py --steps 30 --warmup 5 --no-cpu --no-extras --precision bf16 > $O/prof16.log 2>&1 || { tail -30 $O/prof16.log; exit 1; }
python tools/step_timeline.py $(find $O/prof16 -name '*.db' | head -1) > $O/timeline_bf16.txt; tail -3 $O/timeline_bf16.txt
KB="${KB:-pair_d1_vm pair_d0_vm rowsub_e1_vm rowsub_e2_vm rowsub_e3_vm fwd_d1_vm fwd_d0_up fwd_e1_vm bneck}" OUT=$O/sq bash tools/pmc_sq.sh > $O/sq.log 2>&1 || { tail -30 $O/sq.log; exit 1; }
echo sq done
