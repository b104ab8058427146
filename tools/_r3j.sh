set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3j; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_fused_gpu.py tests/test_sx_graph_gpu.py tests/test_parity_gpu.py tests/test_tiny_gpu.py tests/test_variants_gpu.py tests/test_runtime_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 120 python bench.py --workload c1 --no-cpu-baseline --no-kernel-events > $O/c1_$i.log 2>&1 || exit $?
echo "c1 $(tail -1 $O/c1_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["converged_iterations"], d["time_to_tolerance_s"], d["config"]["setup_s"])')"
done
