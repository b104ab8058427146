set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r2zv; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tiny_gpu.py tests/test_fused_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/exp_tiny.py > $O/exp_tiny.log 2>&1; rc=$?; cat $O/exp_tiny.log; exit $rc
