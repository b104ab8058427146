set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r2zz2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_edge_cases_gpu.py tests/test_parity_gpu.py tests/test_dropin_cp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/exp_pad.py PFDR_PAD_ENDS > $O/exp_ends.log 2>&1; rc=$?; cat $O/exp_ends.log; exit $rc
