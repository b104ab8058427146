set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r2m; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_coop_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in "PFDR_COOP=0" "PFDR_COOP=100000" "PFDR_COOP=100000 PFDR_COOP_G=64" "PFDR_COOP=100000 PFDR_COOP_G=32" "PFDR_COOP=100000 PFDR_COOP_G=16"; do
  env $cfg timeout -k 10 120 python bench.py --workload c1 --no-cpu-baseline > $OUT/c1.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('$OUT/c1.log').read().strip().splitlines()[-1]);print('$cfg', d['ms_per_step'], d.get('time_to_tolerance_s'), d['converged_iterations'])"
done
