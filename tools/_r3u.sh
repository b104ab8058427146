set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3u; mkdir -p $O
timeout -k 10 300 python -u tools/exp_sx_lifecycle.py > $O/sx_lifecycle.log 2>&1 || exit $?
cat $O/sx_lifecycle.log
