set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-r4k}; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r4k} tools/gpu_tests.sh "tests/test_seqsum_gpu.py tests/test_seqdif_gpu.py" "tests/test_partition_gpu.py -k seq" || exit 1
timeout -k 10 300 python tools/seqsum_bench.py > $OUT/seqsum.log 2>&1 || exit 1
cat $OUT/seqsum.log
timeout -k 10 300 python bench.py --workload headline_conv --no-cpu-baseline > $OUT/conv.log 2>&1 || exit 1
tail -c 300 $OUT/conv.log; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --workload headline_conv --no-cpu-baseline > $OUT/conv_trace.log 2>&1 || exit 1
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python tools/trace_overlap.py $T k_mono_walk k_edge_sweep_tl
python tools/trace_overlap.py $T k_mono_walk k_vertex_sweep
S=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
python - "$S" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-40s %6s %9.1f us" % (r["Name"][:40], r["Calls"], float(r["AverageNs"])/1e3))
PY
