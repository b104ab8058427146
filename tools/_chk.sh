set -u
O=gpurun_out/gram1
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gram_gpu.py tests/test_abi.py -m gpu -q -x -s > $O/pytest.log 2>&1; rc=$?
grep -E "gram |opnorm|passed|failed|Error|assert" $O/pytest.log | head -60 | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload c3 > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
tail -1 $O/c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['extra'], d['roofline']['kernels_mean_ms'])"
