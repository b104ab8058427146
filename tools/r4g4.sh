set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r4g4; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_line.log 2>&1 || exit 1
tail -c 300 $OUT/driver_line.log; echo
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -2 $OUT/smoke.log
