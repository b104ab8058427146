set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r4zc; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 150 --warmup 0 --no-cpu-baseline --no-kernel-events > $OUT/b.log 2>&1 || exit 1
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 tools/iter_profile.py $T
