set -u
O=gpurun_out/xcd2
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "simplex" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for x in 00 10 11; do
PFDR_SX_XCD=$x timeout -k 10 300 python bench.py --workload c4 > $O/c4_$x.log 2>&1 || exit 1
tail -1 $O/c4_$x.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 $x', d['ms_per_step'], d['roofline']['kernels_mean_ms'])"
done
