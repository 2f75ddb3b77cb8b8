#!/bin/bash
# Device time (rocprofv3 kernel trace, avg per dispatch) of kbench cases under
# several environment settings of the product library (A/B of runtime knobs).
# usage: KB="fwd_d0 fwd_d1" ENVS="CFSD_KS=0 CFSD_KS=9:1 CFSD_KS=3:2" OUT=gpurun_out/kbe bash tools/kb_env.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/kbe}
rm -rf $OUT; mkdir -p $OUT
export KB_ITERS=${KB_ITERS:-30}
i=0
for e in ${ENVS:-none}; do
  i=$((i+1))
  echo "== $e" | tee -a $OUT/all.log
  if [ "$e" = none ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/v$i -o kb -- python3 tools/kbench.py ${KB:-fwd_d0} > $OUT/v$i.log 2>&1
  else
    export "$e"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/v$i -o kb -- python3 tools/kbench.py ${KB:-fwd_d0} > $OUT/v$i.log 2>&1
    unset "${e%%=*}"
  fi
  python tools/prof_summary.py $(find $OUT/v$i -name '*.db' | head -1) 40 | grep cfsd | cut -c1-150 | tee -a $OUT/all.log
done
