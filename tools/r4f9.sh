set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r4f9; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 tools/devin_check.py headline c1 c2 c4 headline_shuffled || exit 1
for v in dev host dev host; do
  X=""; [ $v = host ] && X="--host-inputs"
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $X > $OUT/d_$v.log 2>&1 || exit 1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/d_$v.log) $(grep -o '"setup_s": [0-9.]*' $OUT/d_$v.log) $(grep -o '"device_inputs": [a-z]*' $OUT/d_$v.log)"
done
