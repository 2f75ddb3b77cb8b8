# coarse dW body rewrite: parity + kernel A/B vs variants/libcfsd_base.so + step A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r7d}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_vm32.py tests/test_gpu_bf16.py tests/test_c4_body.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
KB="${KB:-pair_d1_vm pair_d0_vm rowsub_e1_vm rowsub_e2_vm rowsub_e3_vm}" PAT="${PAT:-lat_pair|ks_pair|lds_pair|flat_pair|rowsub_pair|reduce}" OUT=$O/abk bash tools/ab_kernel.sh > $O/abk.txt 2>&1 || { tail -20 $O/abk.txt; exit 1; }
cat $O/abk.txt
AB_ENVS="CFSD_LIB_PATH=$PWD/variants/libcfsd_base.so;NONE=0" bash tools/ab_bench.sh > $O/abb.txt 2>&1 || { tail -20 $O/abb.txt; exit 1; }
cat $O/abb.txt
AB_ARGS="--precision bf16" AB_ENVS="CFSD_LIB_PATH=$PWD/variants/libcfsd_base.so;NONE=0" bash tools/ab_bench.sh > $O/abb16.txt 2>&1 || { tail -20 $O/abb16.txt; exit 1; }
cat $O/abb16.txt
