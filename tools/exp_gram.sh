# Gram kernel A/B: CFGS="PFDR_GRAM_WIDE=0,PFDR_GRAM_WIDE=1;PFDR_GRAM_TARGET=1280"
# (comma separates configs, ';' joins vars); prints gram kernel ms for c3 and c3_ata
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-gram}; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for cfg in $(echo ${CFGS:-base} | tr ',' ' '); do
  i=$((i+1)); envs=$(echo $cfg | tr ';' ' '); [ "$cfg" = base ] && envs=""
  for wl in c3 c3_ata; do
    env $envs timeout -k 10 300 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > $OUT/${wl}_$i.log 2>&1 || exit $?
    python -c "import json;d=json.loads(open('$OUT/${wl}_$i.log').read().strip().splitlines()[-1]);e=d['extra'];g=e.get('gram') or e.get('operator_norm');print('$cfg', '$wl', g.get('kernel_ms', g.get('gram_kernel_ms')))"
  done
done
