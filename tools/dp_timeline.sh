# Host gaps of the data-parallel step structure (three graph replays around
# the two all-reduce buckets) on ONE GPU with a loopback averager
# (tools/dp_gaps.py): wall time per step vs the single-GPU graph, then the
# kernel timeline of one steady-state step with its gaps (tools/dp_timeline.py).  usage (via gpurun): TAG=round5d bash tools/dp_timeline.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-round5}; mkdir -p $O
timeout -k 10 240 python3 tools/dp_gaps.py 400 > $O/dp_gaps.txt 2>&1 && cat $O/dp_gaps.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_dp -o dp -- python3 tools/dp_gaps.py 40 > $O/dp_prof.log 2>&1
python tools/dp_timeline.py $(find $O/prof_dp -name '*.db' | head -1) > $O/dp_timeline.txt
rm -rf $O/prof_dp
cat $O/dp_timeline.txt
