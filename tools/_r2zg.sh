set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r2zg; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
for wl in c2 c5 headline; do timeout -k 10 400 python bench.py --workload $wl --no-cpu-baseline > $O/bench_$wl.log 2>&1 || exit $?; echo "$wl $(tail -1 $O/bench_$wl.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["mean_ms"], d["roofline"]["frac"], d["roofline"]["kernel"])')"; done
TAG=r2zg WL=c4 E=19985370 V=4999696 bash tools/profile.sh > $O/prof_c4.log 2>&1 || exit $?
echo c4 profiled
