set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3q; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_sx_graph_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
PFDR_SX_V2=1 timeout -k 10 800 python -u -m pytest tests/test_parity_gpu.py tests/test_partition_gpu.py tests/test_dropin_cp.py -m gpu -x -q --timeout 300 --timeout-method thread -k "simplex or sx or dropin" > $O/pytest_v2.log 2>&1; rc=$?
echo "pytest v2 rc=$rc $(tail -1 $O/pytest_v2.log)"; [ $rc -ne 0 ] && exit $rc
TAG=r3q WLS="c4" CFGS="base,PFDR_SX_V2=1,base,PFDR_SX_V2=1" bash tools/ab_wl_env.sh
