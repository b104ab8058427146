set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-r4w}; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r4w} tools/gpu_tests.sh "tests/test_fullsize_gpu.py tests/test_partition_tiled_gpu.py" "tests/test_fullsize_pin_gpu.py -k 'not c5'" || exit 1
for w in headline c2 c5; do
  for v in rec norec rec; do
    if [ $v = norec ]; then export PFDR_LIB_PATH=scratch/norec.so; else unset PFDR_LIB_PATH; fi
    timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $OUT/${w}_$v.log 2>&1 || exit 1
    echo "$w $v $(grep -o '"ms_per_step": [0-9.]*' $OUT/${w}_$v.log) $(grep -o '"kernels_mean_ms": {[^}]*}' $OUT/${w}_$v.log) $(grep -o '"record_blocks": [0-9]*' $OUT/${w}_$v.log)"
  done
done
