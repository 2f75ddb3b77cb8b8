# One GPU-box pass made of named steps, each under its own time limit, stopping at the first failure.
# usage (via gpurun): TAG=round5a bash tools/gpu_steps.sh tests bench prof32 prof16 bench16 pmc32 pmc16 smoke
#   PYTEST_K / PYTEST_FILES narrow the tests step; BENCH_ARGS is appended to the bench steps.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-round5}; mkdir -p $O
for s in ${*:-tests bench prof32}; do
  echo "== $s $(date +%T)"
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests} -x -v -m gpu --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head -20; tail -60 $O/tests.log; exit 1; }
      tail -2 $O/tests.log ;;
    bench)
      timeout -k 10 400 python bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
      cut -c1-600 $O/bench.json; echo ;;
    bench16)
      timeout -k 10 300 python bench.py --precision bf16 --no-cpu --steps 2000 ${BENCH_ARGS} > $O/bench_bf16.json 2> $O/bench_bf16.err || { tail -30 $O/bench_bf16.err; exit 1; }
      cut -c1-600 $O/bench_bf16.json; echo ;;
    prof32|prof16)
      P=fp32; [ $s = prof16 ] && P=bf16
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$P -o bench -- python3 bench.py --precision $P --steps 30 --warmup 5 --no-cpu --no-extras > $O/prof_$P.log 2>&1 || { tail -30 $O/prof_$P.log; exit 1; }
      python tools/step_timeline.py $(find $O/prof_$P -name '*.db' | head -1) > $O/timeline_$P.txt
      python tools/prof_summary.py $(find $O/prof_$P -name '*.db' | head -1) 60 > $O/kernel_stats_$P.txt
      rm -rf $O/prof_$P
      cat $O/timeline_$P.txt ;;
    pmc32)
      CASES="fwd_d3_vm:conv_fwd_vm32<32, 32, 1, 2, 1>:conv_fwd_d3_vm dxf_d3_vm:conv_dx_flat_vm32<32, 32, 16, float>:conv_dx_d3_vm dw_d3_vm:conv_dw_vm32:conv_dw_d3_vm" OUT=$O/traffic32 TAG=$TAG bash tools/pmc_traffic.sh > /dev/null
      cat $O/traffic32/*.json ;;
    pmc16)
      CASES="fwd_d3_b16:conv_fwd_vm16<32, 32, 1, unsigned short>:conv_fwd_d3_bf16_vm dxf_d3_b16:conv_dx_flat_vm16<32, 32, unsigned short, 16>:conv_dx_d3_bf16_vm dw_d3_b16:conv_dw_vm16<unsigned short>:conv_dw_d3_bf16_vm pair_d3_b16:conv_bwd_vm16_pair<16>:conv_pair_d3_bf16_vm" OUT=$O/traffic16 TAG=$TAG bash tools/pmc_traffic.sh > /dev/null
      cat $O/traffic16/*.json ;;
    pmc0)  # the level-0 bandwidth kernels: up0 transpose, output-conv forward / backward
      CASES="spmm_up0T_vm:spmm_sched_csr_k:spmm_up0T_vm dout_fwd_vm:conv_fwd_out_vm:conv_out_fwd_vm dout_bwd_flat:conv_bwd_out_vm:conv_out_bwd_vm spmm_up0T_b16:spmm_sched_csr_k<unsigned short, unsigned short, 8, true>:spmm_up0T_bf16_vm" OUT=$O/traffic0 TAG=$TAG bash tools/pmc_traffic.sh > /dev/null
      cat $O/traffic0/*.json ;;
    kbench)
      timeout -k 10 300 python tools/kbench.py ${KB_CASES} > $O/kbench.txt 2>&1 || { tail -30 $O/kbench.txt; exit 1; }
      cat $O/kbench.txt ;;
    kprof)  # kbench cases under a kernel trace: per-kernel device time (KPROF_ENVS: "A=1 B=2;C=3" variants)
      IFS=';' read -ra VARS <<< "${KPROF_ENVS:-NONE=0}"
      i=0
      for v in "${VARS[@]}"; do
        i=$((i+1))
        env $v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kprof$i -o kb -- python3 tools/kbench.py ${KB_CASES} > $O/kprof$i.log 2>&1 || { tail -20 $O/kprof$i.log; exit 1; }
        echo "-- variant $v" >> $O/kprof.txt
        python tools/prof_summary.py $(find $O/kprof$i -name '*.db' | head -1) 40 >> $O/kprof.txt
        rm -rf $O/kprof$i
      done
      grep -v "at::native\|rocclr\|distribution_elementwise" $O/kprof.txt ;;
    sq)
      KB="${SQ_CASES}" OUT=$O/sq bash tools/pmc_sq.sh > /dev/null
      cat $O/sq/summary.txt ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
      tail -2 $O/smoke.log ;;
  esac
done
