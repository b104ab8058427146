set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${TAG:-r4v} PMC_WL="c2 c4 c5" bash tools/measure.sh pmc cnt || exit 1
