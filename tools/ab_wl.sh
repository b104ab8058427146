#!/bin/bash
# A/B of environment knobs on one bench workload (single GPU), paired runs.
#   WL=c4 CFGS="base,PFDR_SX_XCD_CHUNK=64,..." TAG=x bash tools/ab_wl.sh
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-abwl}; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for cfg in $(echo ${CFGS:-base} | tr ',' ' '); do
  i=$((i+1))
  envs=$(echo $cfg | tr ';' ' ')
  [ "$cfg" = base ] && envs=""
  env $envs timeout -k 10 300 python bench.py --workload ${WL:-headline} --no-cpu-baseline ${BENCH_EXTRA:-} > $OUT/bench_$i.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('$OUT/bench_$i.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$cfg', d['ms_per_step'], d['value'], r['kernel'], r['mean_ms'], r.get('kernels_mean_ms'))"
done
