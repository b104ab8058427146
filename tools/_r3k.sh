set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3k; mkdir -p $O
for e in 1 0; do
PFDR_PAD_ENDS=$e timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c1_$e -o run --output-format csv -- python bench.py --workload c1 --no-cpu-baseline --no-kernel-events > $O/c1_$e.log 2>&1 || exit $?
python tools/trace_gaps.py $O/c1_$e/run_kernel_trace.csv 1500 > $O/gaps_$e.txt
echo "ends=$e"; sed -n 1,5p $O/gaps_$e.txt
done
