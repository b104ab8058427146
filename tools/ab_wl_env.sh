# A/B of environment knobs across workloads (single GPU).
# WLS="headline c2 ..."  CFGS="base,NAME=VAL;NAME=VAL,..." (comma separates configs, ';' joins vars)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-abwl}; mkdir -p $OUT; export TMPDIR=/tmp
for wl in ${WLS:-headline}; do
  i=0
  for cfg in $(echo ${CFGS:-base} | tr ',' ' '); do
    i=$((i+1))
    envs=$(echo $cfg | tr ';' ' ')
    [ "$cfg" = base ] && envs=""
    env $envs timeout -k 10 400 python bench.py --workload $wl ${STEPS:+--steps $STEPS} --no-cpu-baseline ${BENCH_EXTRA:-} > $OUT/${wl}_$i.log 2>&1 || exit $?
    python -c "import json;d=json.loads(open('$OUT/${wl}_$i.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$wl', '$cfg', d['ms_per_step'], 'dom', r['mean_ms'], r.get('kernels_mean_ms'), r['frac'])"
  done
done
