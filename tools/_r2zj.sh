set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r2zj; mkdir -p $O
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
B="python bench.py --workload c4 --no-cpu-baseline --steps 3 --warmup 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_BUSY_CYCLES -d $O/sq -o run --output-format csv -- $B > $O/sq.log 2>&1; echo "sq rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TA_BUSY_avr TA_BUSY_max -d $O/ta -o run --output-format csv -- $B > $O/ta.log 2>&1; echo "ta rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $B > $O/fetch.log 2>&1; echo "fetch rc=$?"
exit 0
