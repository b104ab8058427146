# A/B of environment knobs on the headline bench (single GPU).
# CFGS="NAME=VAL;NAME=VAL,NAME=VAL,..."  (comma separates configs, ';' joins vars)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT; export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x > $OUT/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"; [ $rc -le 1 ] || exit $rc
fi
i=0
for cfg in $(echo ${CFGS:-base} | tr ',' ' '); do
  i=$((i+1))
  envs=$(echo $cfg | tr ';' ' ')
  [ "$cfg" = base ] && envs=""
  env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline ${BENCH_EXTRA:-} > $OUT/bench_$i.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('$OUT/bench_$i.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$cfg', d['ms_per_step'], d['value'], 'edge', r['mean_ms'], 'vertex', r.get('kernels_mean_ms', {}).get('vertex_sweep'), r['frac'], 'chunks', d['config'].get('pipeline_chunks'))"
done
