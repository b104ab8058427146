set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r4f3; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/c1 -o run --output-format csv -- python3 bench.py --workload c1 --no-cpu-baseline --no-kernel-events > $OUT/c1.log 2>&1 || exit 1
T=$(find $OUT/c1 -name "*kernel_trace.csv" | head -1)
python3 tools/trace_gaps.py $T 300 | head -30
