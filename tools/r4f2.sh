set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r4f2; mkdir -p $OUT
TAG=r4f2 LIMIT=700 tools/gpu_tests.sh "tests -p no:randomly" || exit 1
TAG=r4f2 tools/measure.sh bench conv wl || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -3 $OUT/smoke.log
