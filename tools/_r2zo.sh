set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r2zo; mkdir -p $O


for i in 1 2; do
for p in 1 0; do
PFDR_PAD=$p timeout -k 10 120 python bench.py --workload c1 --no-cpu-baseline --no-kernel-events > $O/c1_pad${p}_${i}.log 2>&1 || exit $?
echo "pad=$p $(tail -1 $O/c1_pad${p}_${i}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["converged_iterations"], d["time_to_tolerance_s"])')"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c1 -o run --output-format csv -- python bench.py --workload c1 --no-cpu-baseline --no-kernel-events > $O/c1.log 2>&1 || exit $?
python tools/trace_gaps.py $(ls $O/c1/*kernel_trace.csv | head -1) 1500 | tee $O/c1_gaps.txt
