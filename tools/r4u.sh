set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${TAG:-r4u} LIMIT=700 tools/gpu_tests.sh "tests -p no:randomly" || exit 1
TAG=${TAG:-r4u} tools/measure.sh bench conv wl || exit 1
