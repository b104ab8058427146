set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r2zn; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c1 -o run --output-format csv -- python bench.py --workload c1 --no-cpu-baseline --no-kernel-events > $O/c1.log 2>&1 || exit $?
tail -1 $O/c1.log
python tools/trace_gaps.py $(ls $O/c1/*kernel_trace.csv | head -1) 1500 | tee $O/c1_gaps.txt
