set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3m; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_sx_graph_gpu.py tests/test_parity_gpu.py tests/test_dropin_cp.py tests/test_edge_cases_gpu.py tests/test_partition_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python tools/exp_sx_small.py PFDR_SX_TINY 100000000 > $O/exp_sx_tiny.log 2>&1; rc=$?; cat $O/exp_sx_tiny.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --workload c4 --no-cpu-baseline > $O/c4.log 2>&1 || exit $?
tail -1 $O/c4.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c4", d["ms_per_step"], d["roofline"]["kernels_mean_ms"])'
