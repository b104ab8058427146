set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r2zw; mkdir -p $O
timeout -k 10 400 python tools/exp_tiny.py > $O/exp_tiny_old.log 2>&1; rc=$?; cat $O/exp_tiny_old.log; exit $rc
