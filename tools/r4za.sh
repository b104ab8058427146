set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r4za; mkdir -p $OUT; export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/d_$i.log 2>&1 || exit 1
  echo "d$i $(grep -o '"ms_per_step": [0-9.]*' $OUT/d_$i.log) $(grep -o '"kernels_mean_ms": {[^}]*}' $OUT/d_$i.log) $(grep -o '"cpu_baseline": {"value": [0-9.]*' $OUT/d_$i.log)"
done
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > $OUT/s50.log 2>&1 || exit 1
echo "s50 $(grep -o '"ms_per_step": [0-9.]*' $OUT/s50.log)"
timeout -k 10 300 python3 bench.py --workload headline_conv --no-cpu-baseline > $OUT/conv.log 2>&1 || exit 1
echo "conv $(grep -o '"ms_per_step": [0-9.]*' $OUT/conv.log)"
