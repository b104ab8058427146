set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r2zt; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cp_graph_gpu.py tests/test_segmono_gpu.py tests/test_dropin_cp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
PFDR_BFS_HOST=1 timeout -k 10 600 python -u -m pytest tests/test_cp_graph_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_host.log 2>&1; rc=$?
echo "pytest (host BFS) rc=$rc $(tail -1 $O/pytest_host.log)"; [ $rc -ne 0 ] && exit $rc
for m in 0 1; do
PFDR_BFS_HOST=$m timeout -k 10 300 python tools/bench_cpgraph.py > $O/bench_cpgraph_host$m.log 2>&1 || exit $?
tail -1 $O/bench_cpgraph_host$m.log | cut -c1-520
done
