#!/bin/bash
# Parity tests + kernel-trace stats of tools/kbench.py cases on the GPU box.
# usage: KB="fwd_d3 dx_d3" TESTK=conv bash tools/kb_prof.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/kb}
rm -rf $OUT; mkdir -p $OUT
if [ -n "${TESTK}" ]; then
  timeout -k 10 500 python -m pytest tests/ -x -q -m gpu -k "${TESTK}" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
fi
export KB_ITERS=${KB_ITERS:-50}
timeout -k 10 300 python tools/kbench.py ${KB:-fwd_d3} > $OUT/kb_events.log 2>&1 && cat $OUT/kb_events.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kb -- python tools/kbench.py ${KB:-fwd_d3} > $OUT/kb.log 2>&1
python tools/prof_summary.py $(find $OUT/prof -name '*.db' | head -1) 30
