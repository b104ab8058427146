set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r2zq; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_tiny_gpu.py tests/test_coop_gpu.py tests/test_edge_cases_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/exp_pad.py > $O/exp_pad.log 2>&1; rc=$?; cat $O/exp_pad.log; exit $rc
