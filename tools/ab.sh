#!/bin/bash
# Paired A/B of the in-tree library against other builds of it on one GPU
# box: correctness of the in-tree build first (TESTS, default the tiled and
# full-size pin tests), then bench.py per workload over the ARMS (name:library,
# an empty library = the in-tree build; default prev:scratch/prev.so new:),
# ROUNDS times.  Logs under gpurun_out/$TAG/.
#   TAG=r3m WL="headline c2" ARMS="a:scratch/a.so b:" bash tools/ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${TESTS-tests/test_tiled_gpu.py tests/test_fullsize_pin_gpu.py}" ]; then
    timeout -k 10 600 python -u -m pytest ${TESTS-tests/test_tiled_gpu.py tests/test_fullsize_pin_gpu.py} \
        -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
    rc=$?
    tail -n 3 "$OUT/pytest.log"
    [ $rc -eq 0 ] || exit $rc
fi
for w in ${WL:-headline}; do
    for r in $(seq ${ROUNDS:-2}); do
        for al in ${ARMS:-prev:scratch/prev.so new:}; do
            arm=${al%%:*}; L=${al#*:}
            PFDR_LIB_PATH=$L timeout -k 10 ${LIMIT:-300} python bench.py --no-cpu-baseline \
                --workload $w ${BENCH_EXTRA:-} > "$OUT/${arm}_${w}_$r.log" 2>&1 || exit $?
            python - "$OUT/${arm}_${w}_$r.log" $arm $w <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["roofline"]["kernels_mean_ms"]
print("%-5s %-18s %.4f ms/iter  %s" % (sys.argv[2], sys.argv[3], d["ms_per_step"],
      "  ".join("%s %.4f" % (a, b) for a, b in k.items())))
EOF
        done
    done
done
exit 0
