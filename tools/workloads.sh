#!/bin/bash
# BASELINE.json configs C1..C5 on one GPU (bench.py --workload), one process
# each under its own time limit; stops at the first failure.  Logs under
# gpurun_out/$TAG/.  WL="c1 c2" selects a subset.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-wl}
mkdir -p "$OUT"
export TMPDIR=/tmp
for w in ${WL:-c1 c2 c3 c4 c5}; do
    t0=$(date +%s)
    timeout -k 10 "${LIMIT:-400}" python bench.py --workload "$w" > "$OUT/$w.log" 2>&1
    rc=$?
    echo "[$w] rc=$rc $(( $(date +%s) - t0 ))s"
    tail -n 1 "$OUT/$w.log"
    [ $rc -eq 0 ] || exit $rc
done
exit 0
