set -u
O=gpurun_out/rw1
mkdir -p $O
PFDR_EDGE_RW=1 timeout -k 10 900 python -m pytest tests -m gpu -q -x -k "not gram" > $O/pytest_rw.log 2>&1; rc=$?
grep -E "passed|failed|Error|assert" $O/pytest_rw.log | tail -10 | cut -c1-300
[ $rc -eq 0 ] || exit $rc
for rw in 0 1 0 1; do
PFDR_EDGE_RW=$rw timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > $O/h_$rw.log 2>&1 || exit 1
tail -1 $O/h_$rw.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rw=$rw', d['ms_per_step'], d['roofline']['kernels_mean_ms'], d['config']['device_bytes'])"
done
for rw in 0 1; do
PFDR_EDGE_RW=$rw timeout -k 10 300 python bench.py --workload c2 > $O/c2_$rw.log 2>&1 || exit 1
tail -1 $O/c2_$rw.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 rw=$rw', d['ms_per_step'], d['roofline']['kernels_mean_ms'])"
PFDR_EDGE_RW=$rw timeout -k 10 300 python bench.py --workload c1 > $O/c1_$rw.log 2>&1 || exit 1
tail -1 $O/c1_$rw.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1 rw=$rw', d['ms_per_step'], d['converged_iterations'], d['roofline']['kernels_mean_ms'])"
done
