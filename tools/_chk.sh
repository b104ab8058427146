set -u
O=gpurun_out/fs1
mkdir -p $O
timeout -k 10 1000 python -m pytest tests -m gpu -q -x --durations=8 > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|Error|assert|s call" $O/pytest.log | tail -20 | cut -c1-200
exit $rc
