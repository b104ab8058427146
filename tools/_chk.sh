set -u
O=gpurun_out/cpr1
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_cp_reduce.py tests/test_frontend.py tests/test_abi.py -m gpu -q -x > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|Error|assert" $O/pytest.log | tail -20 | cut -c1-300
exit $rc
