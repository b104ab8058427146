# rocprofv3 kernel stats + PMC traffic (FETCH_SIZE and WRITE_SIZE in separate
# passes, kernel trace only) of one bench workload; summaries -> $OUT.
#   TAG=r1o WL=headline E=60000000 V=10000000 bash tools/profile.sh
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-prof}_${WL:-headline}; mkdir -p $OUT; export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --workload ${WL:-headline} ${BENCH_EXTRA:-}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $B --steps 20 --warmup 3 > $OUT/stats.log 2>&1 || exit $?
echo "stats ok"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B --steps 5 --warmup 1 > $OUT/fetch.log 2>&1 || exit $?
echo "fetch ok"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B --steps 5 --warmup 1 > $OUT/write.log 2>&1 || exit $?
echo "write ok"
python tools/pmc_traffic.py $OUT ${WL:-headline} ${E:-60000000} ${V:-10000000} > $OUT/pmc_traffic.json && cp $OUT/pmc_traffic.json gpurun_out/pmc_${WL:-headline}.json && cat $OUT/pmc_traffic.json
