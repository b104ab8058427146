set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r4j; mkdir -p $OUT; export TMPDIR=/tmp
TAG=r4j tools/gpu_tests.sh "tests/test_seqdif_gpu.py tests/test_sx_graph_gpu.py tests/test_parity_gpu.py -k simplex" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python bench.py --workload headline_conv --no-cpu-baseline > $OUT/conv_trace.log 2>&1 || exit 1
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python tools/trace_overlap.py $T k_mono_ k_edge_sweep_tl
python tools/trace_overlap.py $T k_mono_walk k_edge_sweep_tl
python tools/trace_overlap.py $T k_mono_ k_vertex_sweep
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline > $OUT/c4.log 2>&1 || exit 1
tail -c 600 $OUT/c4.log
