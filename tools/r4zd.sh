set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r4zd; mkdir -p $OUT; export TMPDIR=/tmp
TAG=r4zd tools/gpu_tests.sh "tests/test_fullsize_pin_gpu.py -k 'not c5 and not partitioned'" || exit 1
for v in select branch; do
  if [ $v = branch ]; then export PFDR_LIB_PATH=scratch/branch.so; else unset PFDR_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace_$v -o run --output-format csv -- python3 bench.py --steps 150 --warmup 0 --no-cpu-baseline --no-kernel-events > $OUT/b_$v.log 2>&1 || exit 1
  T=$(find $OUT/trace_$v -name "*kernel_trace.csv" | head -1)
  echo "== $v"; python3 tools/iter_profile.py $T
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/d_$v.log 2>&1 || exit 1
  echo "$v d20 $(grep -o '"ms_per_step": [0-9.]*' $OUT/d_$v.log)"
done
