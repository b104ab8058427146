# headline bench with and without per-kernel HIP events in the timed region
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-events}; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for mode in events bare; do
    extra=""; [ $mode = bare ] && extra="--no-kernel-events"
    timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline $extra ${BENCH_EXTRA:-} > $OUT/bench_${mode}_$rep.log 2>&1 || exit $?
    python -c "import json;d=json.loads(open('$OUT/bench_${mode}_$rep.log').read().strip().splitlines()[-1]);print('$mode rep=$rep', d['ms_per_step'], d['value'], d['roofline']['kernels_mean_ms'])"
  done
done
