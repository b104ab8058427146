set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-r4s}; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r4s} tools/gpu_tests.sh "tests/test_fullsize_gpu.py tests/test_partition_tiled_gpu.py tests/test_erec_gpu.py" "tests/test_fullsize_pin_gpu.py -k 'not c5'" || exit 1
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1 || exit 1
tail -c 1500 $OUT/bench.log; echo
TAG=${TAG:-r4s} PMC_WL=headline bash tools/measure.sh pmc || exit 1
