set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/${TAG:-r2zi}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -k "simplex or sx or partition or dropin" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline > $O/c4_$i.log 2>&1 || exit $?
  tail -1 $O/c4_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernels_mean_ms"])'
done
