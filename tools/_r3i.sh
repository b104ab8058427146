set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3i; mkdir -p $O
run() { timeout -k 10 400 python bench.py "$@" > $O/b.log 2>&1 || exit $?; echo "$* -> $(tail -1 $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernels_mean_ms"])')"; }
run --steps 20 --warmup 5 --no-cpu-baseline
run --steps 20 --warmup 30 --no-cpu-baseline
run --steps 20 --warmup 100 --no-cpu-baseline
run --steps 100 --warmup 5 --no-cpu-baseline
run --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-events
run --steps 20 --warmup 5
