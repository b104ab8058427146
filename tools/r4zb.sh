set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r4zb; mkdir -p $OUT; export TMPDIR=/tmp
run() { timeout -k 10 300 python3 bench.py --gpus 1 --steps ${2:-20} --warmup 5 --no-cpu-baseline > $OUT/$1.log 2>&1 || exit 1
  echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/$1.log) $(grep -o '"kernels_mean_ms": {[^}]*}' $OUT/$1.log) $(grep -o '"setup_s": [0-9.]*' $OUT/$1.log)"; }
run first
run hot1
run hot2
echo "idle 40 s"; sleep 40
run after_idle
run hot3
run hot_s100 100
echo "idle 40 s"; sleep 40
run after_idle_s100 100
