set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r2zs; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_segmono_gpu.py tests/test_cp_graph_gpu.py tests/test_cp_reduce.py tests/test_dropin_cp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
for m in 1 0; do
PFDR_SEGMONO=$m timeout -k 10 300 python tools/bench_cpgraph.py > $O/bench_cpgraph_mono$m.log 2>&1 || exit $?
tail -1 $O/bench_cpgraph_mono$m.log | cut -c1-600
PFDR_SEGMONO=$m timeout -k 10 300 python tools/bench_cpgraph_simplex.py > $O/bench_cpgraph_simplex_mono$m.log 2>&1 || exit $?
tail -1 $O/bench_cpgraph_simplex_mono$m.log | cut -c1-600
done
