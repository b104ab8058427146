set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=r4g3 LIMIT=700 tools/gpu_tests.sh "tests -p no:randomly" || exit 1
TAG=r4g3 PMC_WL="c4" WL="c4" bash tools/measure.sh pmc wl || exit 1
