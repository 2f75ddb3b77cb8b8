# Same-box A/B of the in-tree libcfsd.so against ab_lib/libcfsd_base.so (HEAD's build):
# optional parity tests (TESTK = pytest -k filter), kernel-trace stats of kbench cases
# (KB) under both libraries, then whole-step A/B in fp32 and bf16 (PRECS).
# usage (via gpurun): TAG=r8b TESTK=bottleneck KB="bneck" bash tools/gpu_ab.sh
# BASEDIR=ab_base: the base is a whole tree (HEAD's sources + its library) run from that
# directory -- for changes of the ABI, where only the library cannot be swapped.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-ab}; rm -rf $O; mkdir -p $O
BASE=$GRAFT_REPO_ROOT/ab_lib/libcfsd_base.so
if [ -n "${TESTK}" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "${TESTK}" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
export KB_ITERS=${KB_ITERS:-50}
if [ -n "${KB}" ]; then
  for v in base new; do
    if [ $v = base ]; then L=$BASE; else L=""; fi
    D=$GRAFT_REPO_ROOT; if [ $v = base ] && [ -n "$BASEDIR" ]; then D=$GRAFT_REPO_ROOT/$BASEDIR; L=""; fi
    (cd $D && CFSD_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kb_$v -o kb -- python3 tools/kbench.py ${KB}) > $O/kb_$v.log 2>&1 || { tail -30 $O/kb_$v.log; exit 1; }
    echo "== kbench $v"; grep " us" $O/kb_$v.log || true
    python tools/prof_summary.py $(find $O/kb_$v -name '*.db' | head -1) 12 > $O/kb_stats_$v.txt
    head -14 $O/kb_stats_$v.txt
  done
fi
for p in ${PRECS:-fp32 bf16}; do
  for rep in 1 2; do
    for v in base new; do
      if [ $v = base ]; then L=$BASE; else L=""; fi
      D=$GRAFT_REPO_ROOT; if [ $v = base ] && [ -n "$BASEDIR" ]; then D=$GRAFT_REPO_ROOT/$BASEDIR; L=""; fi
      (cd $D && CFSD_LIB_PATH=$L timeout -k 10 200 python bench.py --no-cpu --no-extras --no-bf16 --steps ${STEPS:-3000} --warmup 50 --precision $p) > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$p rep $rep $v  ms/step %.4f  %.0f meshes/s' % (d['ms_per_step'], d['value']))" | tee -a $O/ab_summary.txt
    done
  done
done
