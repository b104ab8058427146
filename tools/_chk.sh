set -u
O=gpurun_out/ov1
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|Error|assert" $O/pytest.log | tail -20 | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > $O/headline.log 2>&1 || exit 1
tail -1 $O/headline.log | cut -c1-300
