#!/bin/bash
# One GPU-box session: GPU parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fault/abort/timeout stops the
# script (no further GPU work in the call).  Logs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name limit cmd...
    local name=$1 lim=$2; shift 2
    local t0=$(date +%s)
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
    tail -n 3 "$OUT/$name.log"
    return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }   # 1 = test failures only
step pytest_gpu 1200 python -m pytest tests -m gpu -q -rf -s; rc=$?
fatal $rc && exit $rc
[ "${SKIP_SMOKE:-0}" = 1 ] || { step smoke 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" || exit $?; }
[ "${SKIP_BENCH:-0}" = 1 ] || { step bench 900 python bench.py ${BENCH_ARGS:-} || exit $?; }
if [ "${PROFILE:-1}" = 1 ]; then
    step rocprof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
        -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline || exit $?
fi
exit 0
