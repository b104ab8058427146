set -u
O=gpurun_out/sx3
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -q -k "simplex or proj" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
PFDR_SX_WZ=0 timeout -k 10 600 python -m pytest tests -m gpu -q -k "simplex" > $O/pytest_nowz.log 2>&1 || { tail -30 $O/pytest_nowz.log; exit 1; }
tail -2 $O/pytest_nowz.log
for cfg in "PFDR_SX_NT=256" "PFDR_SX_NT=64" "PFDR_SX_WZ=0" "PFDR_SX_WZ=0 PFDR_SX_NT=64"; do
env $cfg timeout -k 10 300 python bench.py --workload c4 > $O/c4.log 2>&1 || exit 1
tail -1 $O/c4.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['ms_per_step'], d['roofline']['kernels_mean_ms'])"
done
