# One GPU-box pass: GPU tests, default bench, rocprofv3 kernel stats + step timeline.
# Usage (from the repo root, via gpurun): TAG=r02a bash tools/gpu_round.sh [tests|bench|prof ...]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r02}; mkdir -p $O
steps="${*:-tests bench prof}"
for s in $steps; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/tests.log 2>&1 || { tail -80 $O/tests.log; exit 1; }
      tail -3 $O/tests.log ;;
    bench)
      timeout -k 10 400 python bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
      cut -c1-400 $O/bench.json ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --steps 30 --warmup 5 --no-cpu --no-extras > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
      python tools/step_timeline.py $(find $O/prof -name '*.db' | head -1) > $O/timeline.txt; tail -60 $O/timeline.txt ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
      tail -2 $O/smoke.log ;;
  esac
done
