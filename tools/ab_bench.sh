# Same-box A/B of whole-step time: AB_ENVS="A=1;B=2" (variants, ';'-separated), run twice interleaved.
# usage (via gpurun): AB_ENVS="X=0;X=1" [AB_ARGS="--precision bf16"] bash tools/ab_bench.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
IFS=';' read -ra VARS <<< "${AB_ENVS:-NONE=0}"
for rep in 1 2; do
  for v in "${VARS[@]}"; do
    env $v timeout -k 10 200 python bench.py --no-cpu --no-extras --steps 3000 --warmup 50 ${AB_ARGS} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('rep $rep  $v  ms/step %.4f  %.0f meshes/s' % (d['ms_per_step'], d['value']))"
  done
done
