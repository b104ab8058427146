#!/bin/bash
# A round's measurement pass on one GPU box, steps chained (a failure stops
# the call): GPU tests named by TESTS, then bench.py over WL (logs under
# gpurun_out/$TAG/), then PMC traffic summaries (tools/profile.sh) for the
# workloads in PMC ("name:E:V" each; summaries under gpurun_out/$TAG_<name>/).
#   TAG=r3z TESTS="tests/test_tiled_gpu.py" WL="headline c2" PMC="c2:50135040:16777216" \
#       bash tools/round_check.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-rc}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
    timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$OUT/pytest.log" 2>&1 || { tail -n 30 "$OUT/pytest.log"; exit 1; }
    tail -n 1 "$OUT/pytest.log"
fi
for w in ${WL:-}; do
    timeout -k 10 ${LIMIT:-400} python bench.py --workload "$w" > "$OUT/$w.log" 2>&1 || exit $?
    python - "$OUT/$w.log" "$w" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print("%-18s %.4f ms/iter  %s frac %s traffic %s  cpu %s" % (sys.argv[2], d["ms_per_step"], r.get("kernel"),
      r.get("frac"), r.get("traffic"), (d.get("cpu_baseline") or {}).get("value")))
PY
done
for spec in ${PMC:-}; do
    IFS=: read -r w e v <<< "$spec"
    TAG=$TAG WL=$w E=$e V=$v bash tools/profile.sh > "$OUT/pmc_$w.log" 2>&1 || { tail -n 5 "$OUT/pmc_$w.log"; exit 1; }
    echo "pmc $w ok"
done
exit 0
