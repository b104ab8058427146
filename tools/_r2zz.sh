set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r2zz; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_tiny_gpu.py tests/test_edge_cases_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/exp_pad.py PFDR_PAD_ENDS > $O/exp_ends.log 2>&1; rc=$?; cat $O/exp_ends.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for p in 1 0; do
PFDR_PAD_ENDS=$p timeout -k 10 120 python bench.py --workload c1 --no-cpu-baseline --no-kernel-events > $O/c1_ends${p}_${i}.log 2>&1 || exit $?
echo "ends=$p $(tail -1 $O/c1_ends${p}_${i}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["converged_iterations"], d["time_to_tolerance_s"])')"
done; done
