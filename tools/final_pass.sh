set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/f6b; mkdir -p $O
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
tail -n 1 $O/bench.log
timeout -k 10 400 python bench.py --gpus 1 --steps 50 --warmup 5 --no-cpu-baseline > $O/bench50.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
echo prof ok
TAG=f6w WL="c1 c2 c3 c3_ata c4 c4k100 c5 headline_conv" bash tools/workloads.sh
