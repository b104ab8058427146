set -u
O=gpurun_out/g2
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -x -s > $O/pytest.log 2>&1; rc=$?
grep -E "^gram|^.gram|passed|failed|Error|assert" $O/pytest.log | tail -30 | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload c3 > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
tail -1 $O/c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['extra'], d['config']['setup_s'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > $O/headline.log 2>&1 || exit 1
tail -1 $O/headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['setup_s'], d['roofline']['kernels_mean_ms'])"
