set -u
O=gpurun_out/ro1
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python bench.py --workload headline_shuffled > $O/shuf.log 2>&1 || { tail -20 $O/shuf.log; exit 1; }
tail -1 $O/shuf.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['setup_s'], d['config']['relabelled'], d['roofline']['kernels_mean_ms'])"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/headline.log 2>&1 || exit 1
tail -1 $O/headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['setup_s'], d['config']['relabelled'], d['roofline']['kernels_mean_ms'])"
