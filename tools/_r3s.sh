set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3s; mkdir -p $O
TAG=r3s WL=headline bash tools/profile.sh > $O/prof_headline.log 2>&1 || exit $?
echo headline profiled
