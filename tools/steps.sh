#!/bin/bash
# One GPU-box session built from named steps, each under its own time limit;
# the first failing step ends the call (no further GPU work after a fault,
# abort or timeout).  Logs under gpurun_out/$TAG/.
#   TAG=r6a STEPS="pytest ab pmc" PYTEST_ARGS="tests/x.py -k 'a or b'" WL=c4 \
#       ARMS="r5:scratch/r5.so new:" bash tools/steps.sh
#   pytest : python -m pytest $PYTEST_ARGS -m gpu (thread timeouts)
#   ab     : bench.py --workload w for every ARM (name:library[:VAR=v,VAR=v], empty library =
#            in-tree), ROUNDS times
#   counters: tools/counters.sh of every WL for every ARM (SQ / TA / LDS counters)
#   pmc    : rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes of every WL (in-tree library,
#            or PMC_LIB), summary gpurun_out/$TAG/pmc_<w>.json
#   bench  : python bench.py $BENCH_ARGS
#   smoke  : __graft_entry__ build() + smoke()
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-steps}
mkdir -p "$OUT"
export TMPDIR=/tmp
line() {
    python - "$1" "$2" "$3" <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
k = r["kernels_mean_ms"]
print("%-5s %-14s %.4f ms/iter  %s  dom=%s frac=%s" % (sys.argv[2], sys.argv[3], d["ms_per_step"],
      "  ".join("%s %.4f" % (a, b) for a, b in k.items()), r.get("kernel"), r.get("frac")))
EOF
}
for st in ${STEPS:-pytest}; do
    t0=$(date +%s)
    case $st in
    pytest)
        eval "timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -x -v -rf \
            --timeout 300 --timeout-method thread" > "$OUT/pytest.log" 2>&1
        rc=$?; tail -n 3 "$OUT/pytest.log" ;;
    ab)
        rc=0
        for w in ${WL:-headline}; do
            for r in $(seq ${ROUNDS:-2}); do
                for al in ${ARMS:-new:}; do
                    arm=${al%%:*}; L=${al#*:}; EV=""
                    case $L in *:*) EV=${L#*:}; L=${L%%:*} ;; esac  # name:lib:VAR=v,VAR=v
                    env ${EV//,/ } PFDR_LIB_PATH=$L timeout -k 10 ${LIMIT:-300} python bench.py --no-cpu-baseline \
                        --workload $w ${BENCH_EXTRA:-} > "$OUT/${arm}_${w}_$r.log" 2>&1 || { rc=$?; break 3; }
                    line "$OUT/${arm}_${w}_$r.log" $arm $w
                done
            done
        done ;;
    pmc)
        rc=0
        for w in ${WL:-headline}; do
            P=$OUT/pmc_$w; mkdir -p $P
            B="python bench.py --no-cpu-baseline --workload $w ${BENCH_EXTRA:-}"
            PFDR_LIB_PATH=${PMC_LIB:-} timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $P/stats -o run \
                --output-format csv -- $B --steps 20 --warmup 3 > $P/stats.log 2>&1 || { rc=$?; break; }
            PFDR_LIB_PATH=${PMC_LIB:-} timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run \
                --output-format csv -- $B --steps 5 --warmup 1 > $P/fetch.log 2>&1 || { rc=$?; break; }
            PFDR_LIB_PATH=${PMC_LIB:-} timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run \
                --output-format csv -- $B --steps 5 --warmup 1 > $P/write.log 2>&1 || { rc=$?; break; }
            python tools/pmc_traffic.py $P $w > $OUT/pmc_$w.json || { rc=$?; break; }
            python - $OUT/pmc_$w.json <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    if v["hbm_bytes_per_launch"] > 1e8:
        print("  %-28s %.3f GB (read %.3f, write %.3f)" % (k, v["hbm_bytes_per_launch"] / 1e9,
              v["read_bytes_per_launch"] / 1e9, v["write_bytes_per_launch"] / 1e9))
EOF
        done ;;
    counters)
        rc=0
        for w in ${WL:-headline}; do
            for al in ${ARMS:-new:}; do
                arm=${al%%:*}; L=${al#*:}; EV=""
                case $L in *:*) EV=${L#*:}; L=${L%%:*} ;; esac
                env ${EV//,/ } PFDR_LIB_PATH=$L TAG=$TAG/cnt_$arm WL=$w bash tools/counters.sh \
                    > "$OUT/cnt_${arm}_$w.log" 2>&1 || { rc=$?; break 2; }
                echo "$arm $w counters ok"
            done
        done ;;
    bench)
        timeout -k 10 ${LIMIT:-600} python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
        rc=$?; tail -n 1 "$OUT/bench.log" ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
        rc=$?; tail -n 2 "$OUT/smoke.log" ;;
    *) echo "unknown step $st"; exit 2 ;;
    esac
    echo "[$st] rc=$rc $(( $(date +%s) - t0 ))s"
    [ $rc -eq 0 ] || exit $rc
done
exit 0
