#!/bin/bash
# What bounds a workload's sweeps: rocprofv3 SQ (wave states, instruction
# mix) and TA (texture addresser busy) counters, one --pmc pass per group,
# kernel trace only; summary per kernel -> $OUT/counters.md.
#   TAG=r3l WL=headline bash tools/counters.sh
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-cnt}_${WL:-headline}; mkdir -p $OUT; export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --workload ${WL:-headline} ${BENCH_EXTRA:-} --steps 5 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD \
    -d $OUT/sq -o run --output-format csv -- $B > $OUT/sq.log 2>&1 || exit $?
echo "sq ok"
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE \
    -d $OUT/ta -o run --output-format csv -- $B > $OUT/ta.log 2>&1 || exit $?
echo "ta ok"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH \
    -d $OUT/sq2 -o run --output-format csv -- $B > $OUT/sq2.log 2>&1 || exit $?
echo "sq2 ok"
python tools/counter_summary.py $OUT > $OUT/counters.md && cat $OUT/counters.md
