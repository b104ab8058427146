set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3n; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_sx_graph_gpu.py tests/test_parity_gpu.py tests/test_dropin_cp.py tests/test_edge_cases_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; exit $rc
