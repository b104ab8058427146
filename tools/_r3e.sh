set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3e; mkdir -p $O
TAG=r3e WL=headline bash tools/profile.sh > $O/prof_headline.log 2>&1 || exit $?
echo headline profiled
cp gpurun_out/r3e_headline/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log
