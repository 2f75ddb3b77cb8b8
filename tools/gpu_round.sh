#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench (+cpu baseline), kernel-trace stats of the bench,
# and HBM-traffic PMC passes (FETCH_SIZE / WRITE_SIZE, one per run) on the dominant kernel.
# usage (from gpurun): bash tools/gpu_round.sh [tag]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
OUT=gpurun_out/$TAG
rm -rf $OUT; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 \
    || { tail -60 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 300 python -u bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --steps 30 --warmup 5 --no-cpu > $OUT/prof.log 2>&1 \
  || { tail -30 $OUT/prof.log; exit 1; }
python tools/prof_summary.py $(find $OUT/prof -name '*.db' | head -1) 60 > $OUT/kernel_stats.txt || true
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \; || true
head -20 $OUT/kernel_stats.txt
if [ -z "$SKIP_PMC" ]; then
  export KB_ITERS=20
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- python3 tools/kbench.py fwd_d3 dx_d3 dw_d3 > $OUT/pmc_fetch.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- python3 tools/kbench.py fwd_d3 dx_d3 dw_d3 > $OUT/pmc_write.log 2>&1
  python tools/pmc_traffic.py $OUT "conv_fwd_mfma<32, 32, 1, 9>" > $OUT/pmc_traffic_conv_fwd_d3.json || true
  python tools/pmc_traffic.py $OUT "conv_dx_mfma<32, 32, 9>" > $OUT/pmc_traffic_conv_dx_d3.json || true
  python tools/pmc_traffic.py $OUT "conv_dw_mfma<32, 32>" > $OUT/pmc_traffic_conv_dw_d3.json || true
  cat $OUT/pmc_traffic_*.json
  KB="fwd_d3 dx_d3 dw_d3" OUT=$OUT/pmc_sq bash tools/pmc_kernels.sh > $OUT/pmc_sq.log 2>&1 || true
  tail -20 $OUT/pmc_sq.log
fi
echo ALL_DONE
