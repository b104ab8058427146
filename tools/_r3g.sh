set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cp_graph_gpu.py tests/test_segmono_gpu.py tests/test_dropin_cp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python tools/bench_cpgraph.py --cpu --reps 3 > $O/bench_cpgraph_cpu.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('$O/bench_cpgraph_cpu.log').read().strip().splitlines()[-1]); print('l1 parity_full_size', d.get('parity_full_size'), d['gpu_ms'], d['gpu_ms_iteration_graph_steps'])"
timeout -k 10 500 python tools/bench_cpgraph_simplex.py --cpu --reps 3 > $O/bench_cpgraph_simplex_cpu.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('$O/bench_cpgraph_simplex_cpu.log').read().strip().splitlines()[-1]); print('simplex', d['gpu_ms'], d['parity_full_size'], d['gpu_ms_iteration_graph_steps'])"
