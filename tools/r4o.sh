set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-r4o}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 scratch/monoprof 10000000 0 || exit 1
TAG=${TAG:-r4o} tools/gpu_tests.sh "tests/test_seqsum_gpu.py tests/test_seqdif_gpu.py" "tests/test_partition_gpu.py -k seq" "tests/test_fullsize_pin_gpu.py -k 'conv and not c5'" "tests/test_parity_gpu.py tests/test_sx_graph_gpu.py -k simplex" || exit 1
timeout -k 10 300 python bench.py --workload headline_conv --no-cpu-baseline > $OUT/conv.log 2>&1 || exit 1
echo "conv $(grep -o 'ms_per_step": [0-9.]*' $OUT/conv.log)"
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python bench.py --workload headline_conv --no-cpu-baseline > $OUT/conv_trace.log 2>&1 || exit 1
