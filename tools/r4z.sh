set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r4z; mkdir -p $OUT; export TMPDIR=/tmp
for v in base upload base upload; do
  if [ $v = upload ]; then export PFDR_LIB_PATH=scratch/upload.so; else unset PFDR_LIB_PATH; fi
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/d_$v.log 2>&1 || exit 1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/d_$v.log) $(grep -o '"kernels_mean_ms": {[^}]*}' $OUT/d_$v.log)"
done
