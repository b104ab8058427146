#!/bin/bash
# One GPU-box call running pytest selections, each under its own limit:
#   TAG=name tools/gpu_tests.sh "sel1" "sel2" ...   (logs: gpurun_out/$TAG/)
# A fault / abort / timeout ends the call (no further GPU step).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-tests}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for sel in "$@"; do
    i=$((i + 1))
    t0=$(date +%s)
    # (eval: a selection may quote a -k expression, e.g. 'tests/x.py -k "a or b"')
    eval timeout -k 10 "${LIMIT:-900}" python -u -m pytest $sel -m gpu -x -v -rf -s \
        --timeout "${TLIMIT:-600}" --timeout-method thread > "$OUT/pytest_$i.log" 2>&1
    rc=$?
    echo "[pytest_$i: $sel] rc=$rc $(( $(date +%s) - t0 ))s"
    tail -n 4 "$OUT/pytest_$i.log"
    [ $rc -ne 0 ] && exit $rc
done
exit 0
