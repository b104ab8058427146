set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sx_fused_gpu.py tests/test_parity_gpu.py tests/test_dropin_cp.py tests/test_partition_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/exp_sx_small.py PFDR_FUSE > $O/exp_sx_fuse.log 2>&1; rc=$?; cat $O/exp_sx_fuse.log; exit $rc
