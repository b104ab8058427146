# A/B of the DR-average variants and the XCD-aware block order.
# CFGS="mode:xcd,mode:xcd,..."  (xcd = <edge bit><vertex bit>)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT; export TMPDIR=/tmp
for m in ${TEST_MODES:-scatter}; do
  PFDR_AVERAGE=$m timeout -k 10 600 python -m pytest tests -m gpu -q -x > $OUT/pytest_$m.log 2>&1; rc=$?
  echo "pytest $m rc=$rc $(tail -1 $OUT/pytest_$m.log)"; [ $rc -le 1 ] || exit $rc
done
for cfg in $(echo ${CFGS:-scatter:01,wz:01} | tr ',' ' '); do
  m=${cfg%%:*}; x=${cfg##*:}
  PFDR_AVERAGE=$m PFDR_XCD=$x timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench_${m}_$x.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('$OUT/bench_${m}_$x.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$m xcd=$x', d['ms_per_step'], d['value'], 'edge', r['mean_ms'], 'vertex', r['vertex_sweep_mean_ms'], r['frac'])"
done
