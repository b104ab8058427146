set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3f; mkdir -p $O
timeout -k 10 500 python tools/bench_cpgraph.py --cpu --reps 3 > $O/bench_cpgraph_cpu.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('$O/bench_cpgraph_cpu.log').read().strip().splitlines()[-1]); print('l1 parity_full_size', d.get('parity_full_size'), d['gpu_ms'])"
timeout -k 10 500 python tools/bench_cpgraph_simplex.py --cpu --reps 3 > $O/bench_cpgraph_simplex_cpu.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('$O/bench_cpgraph_simplex_cpu.log').read().strip().splitlines()[-1]); print('simplex', {k:v for k,v in d.items() if k in ('parity_full_size','ok','gpu_ms','bit_identical')})"
