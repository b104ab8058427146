set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-r4m}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 scratch/monoprof 10000000 0 || exit 1
timeout -k 10 120 scratch/monoprof 10000000 1 || exit 1
TAG=${TAG:-r4m} tools/gpu_tests.sh "tests/test_seqsum_gpu.py tests/test_seqdif_gpu.py" "tests/test_partition_gpu.py -k seq" || exit 1
for v in prio noprio prio; do
  if [ $v = noprio ]; then L=scratch/noprio.so; else L=""; fi
  PFDR_LIB_PATH=$L timeout -k 10 300 python bench.py --workload headline_conv --no-cpu-baseline > $OUT/conv_$v.log 2>&1 || exit 1
  echo "$v $(grep -o 'ms_per_step": [0-9.]*' $OUT/conv_$v.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python bench.py --workload headline_conv --no-cpu-baseline > $OUT/conv_trace.log 2>&1 || exit 1
