set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r4g2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $OUT/clk -o run --output-format csv -- python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-kernel-events > $OUT/b.log 2>&1 || exit 1
python3 tools/clock_trace.py $OUT/clk
