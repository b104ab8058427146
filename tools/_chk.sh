set -u
O=gpurun_out/sxp1
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -k "partition or simplex or proj" > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|Error|error" $O/pytest.log | tail -30 | cut -c1-300
exit $rc
