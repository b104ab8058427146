set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r4f4; mkdir -p $OUT
TAG=r4f4 LIMIT=700 tools/gpu_tests.sh "tests -p no:randomly" || exit 1
for i in 1 2; do
timeout -k 10 300 python3 bench.py --workload c1 --no-cpu-baseline > $OUT/c1_$i.log 2>&1 || exit 1
echo "c1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/c1_$i.log)"
done
