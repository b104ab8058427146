#!/bin/bash
# One GPU call of measurements for DESIGN.md / profiles: the driver's bench
# line, the converged headline, the other BASELINE workloads, rocprofv3
# kernel stats and PMC traffic of the headline.  Every GPU step under its own
# limit; a failure ends the call.  Logs: gpurun_out/$TAG/.
#   TAG=r4d tools/measure.sh [bench] [conv] [conv1r] [wl] [prof] [pmc] [cnt]
# (WL: workloads of `wl`, BENCH_EXTRA: extra bench.py arguments of `wl`)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-meas}; OUT=gpurun_out/$T; mkdir -p "$OUT"; export TMPDIR=/tmp
step() {  # name limit cmd...
    local name=$1 lim=$2; shift 2
    local t0=$(date +%s)
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"; tail -n 1 "$OUT/$name.log" | cut -c1-400
    [ $rc -eq 0 ] || exit $rc
}
for what in "${@:-bench}"; do
  case $what in
    bench) step bench 600 python bench.py ;;
    bench100) step bench100 600 python bench.py --steps 100 --warmup 20 --no-cpu-baseline ;;
    conv) step headline_conv 600 python bench.py --workload headline_conv ;;
    conv1r) step headline_conv_rccl1 600 python bench.py --workload headline_conv \
              --no-cpu-baseline --dist-selftest ;;
    wl) for w in ${WL:-c1 c2 c3 c3_ata c4 c5 headline_shuffled headline_slab8}; do
            step "wl_$w" 600 python bench.py --workload "$w" ${BENCH_EXTRA:-}; done ;;
    prof) step rocprof_stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run \
              --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    pmc) for w in ${PMC_WL:-headline}; do
            TAG=$T WL=$w bash tools/profile.sh > "$OUT/pmc_$w.log" 2>&1 || { tail -5 "$OUT/pmc_$w.log"; exit 1; }
            tail -3 "$OUT/pmc_$w.log"; done ;;
    cnt) TAG=$T WL=headline bash tools/counters.sh > "$OUT/cnt.log" 2>&1 || exit 1; tail -20 "$OUT/cnt.log" ;;
  esac
done
exit 0
