set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3v; mkdir -p $O
timeout -k 10 400 rocprofv3 --hip-runtime-trace --kernel-trace --stats --output-format csv -d $O/prof -o sx -- python3 -u tools/exp_sx_lifecycle.py > $O/run.log 2>&1 || exit $?
find $O/prof -name "*stats*" | head
