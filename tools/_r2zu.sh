set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r2zu; mkdir -p $O
timeout -k 10 300 python tools/bench_cpgraph.py > $O/bench_cpgraph.log 2>&1 || exit $?
tail -1 $O/bench_cpgraph.log | cut -c1-600
