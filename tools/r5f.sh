TAG=round5f PYTEST_FILES="tests/test_gpu_parity.py" PYTEST_K="fused_reduce" bash tools/gpu_steps.sh tests
for m in off final hosts; do
  CFSD_SIDE_MODE=$m timeout -k 10 200 python bench.py --no-cpu --no-extras --steps 5000 > gpurun_out/round5f/bench_$m.json 2>/dev/null && python -c "import json;d=json.load(open('gpurun_out/round5f/bench_$m.json'));print('$m', d['ms_per_step'])"
done
for m in off final hosts; do
  CFSD_SIDE_MODE=$m timeout -k 10 200 python bench.py --no-cpu --no-extras --steps 5000 > gpurun_out/round5f/bench2_$m.json 2>/dev/null && python -c "import json;d=json.load(open('gpurun_out/round5f/bench2_$m.json'));print('$m', d['ms_per_step'])"
done
